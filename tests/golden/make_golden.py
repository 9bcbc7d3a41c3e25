#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (it reads /root/reference, which does not exist
on the GPU box).  Its outputs are data: inputs and expected outputs.

What it does
------------
* Extracts the 1024-entry probability vector of the reference harness
  `benchmark_multiset` (src/multiset.rs:158) and applies the reference's mass
  rule `max(1, (p * 2^28) as usize)` (src/multiset.rs:169-170) -> masses.
  Only the resulting integers are written (masses_multiset.json).
* Copies the reference's fixtures multiset-data/{1000,10000,100000}.txt
  (data files the reference's own test reads, multiset.rs:161-166).
* Encodes them with an INDEPENDENT pure-Python restatement of the reference
  rANS coder (src/ans.rs:96-116,233-264; src/codec.rs:59-69,413-425), written
  separately from oracle/ans_oracle.c, and records the flattened bytes per
  chunk.  The C oracle is checked against these vectors in tests/test_oracle.py.

The reference itself (Rust) cannot be built here, so no
reference-produced byte vectors exist; these fixtures pin the C oracle and the
GPU path to the reference's arithmetic as restated twice.
"""
import hashlib
import json
import math
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
MAX_MIN_HEAD = 1 << 56
MASK64 = (1 << 64) - 1


# ----------------------------------------------------------------------------
# Independent restatement: state = (head, bytes list); zeros generator.
# ----------------------------------------------------------------------------
class Msg:
    def __init__(self, head=MAX_MIN_HEAD, tail=None):
        self.head = head
        self.tail = list(tail or [])
        self.generated = 0

    def _pop_byte(self):
        if self.tail:
            return self.tail.pop()
        self.generated += 1
        return 0  # TailGenerator::Zeros

    def renorm(self, lo):
        # ans.rs:239-253 -- up then down
        while self.head < lo:
            self.head = ((self.head << 8) | self._pop_byte()) & MASK64
        while (self.head >> 8) >= lo:
            self.tail.append(self.head & 0xFF)
            self.head >>= 8

    def flatten(self):
        # ans.rs:255-260
        h, t = self.head, list(self.tail)
        while (h >> 8) >= 1:
            t.append(h & 0xFF)
            h >>= 8
        t.append(h & 0xFF)
        return bytes(t)


def cumulative(masses):
    out, acc = [], 0
    for m in masses:
        out.append(acc)
        acc += m
    return out, acc


def push_sym(msg, masses, cums, norm, x):
    p = masses[x]
    assert p != 0
    msg.renorm(p * (MAX_MIN_HEAD // norm))
    q, r = divmod(msg.head, p)
    msg.head = norm * q + cums[x] + r


def pop_sym(msg, masses, cums, norm):
    msg.renorm(norm * (MAX_MIN_HEAD // norm))
    q, i = divmod(msg.head, norm)
    # last x with cums[x] <= i  (codec.rs:66 partition_point semantics)
    lo, hi = 0, len(cums)
    while lo < hi:
        mid = (lo + hi) // 2
        if cums[mid] <= i:
            lo = mid + 1
        else:
            hi = mid
    x = lo - 1
    msg.head = masses[x] * q + (i - cums[x])
    return x


def encode_chunks(masses, syms, chunk_len):
    cums, norm = cumulative(masses)
    streams = []
    for a in range(0, len(syms), chunk_len):
        m = Msg()
        for x in reversed(syms[a:a + chunk_len]):  # IID pushes in reverse (codec.rs:417)
            push_sym(m, masses, cums, norm, x)
        streams.append(m.flatten())
    return streams


def decode_chunk(masses, stream, count):
    cums, norm = cumulative(masses)
    m = Msg(head=0, tail=list(stream))  # unflatten: head = 0 (ans.rs:262-264)
    out = [pop_sym(m, masses, cums, norm) for _ in range(count)]
    m.renorm(MAX_MIN_HEAD)
    assert m.head == MAX_MIN_HEAD and not m.tail and m.generated == 0, "message did not return to zeros()"
    return out


def info_bits(masses, syms):
    _, norm = cumulative(masses)
    return sum(math.log2(norm) - math.log2(masses[x]) for x in syms)


def record(masses, syms, chunk_len, keep_bytes):
    streams = encode_chunks(masses, syms, chunk_len)
    # self-check: decode every chunk back
    for j, s in enumerate(streams):
        part = syms[j * chunk_len:(j + 1) * chunk_len]
        assert decode_chunk(masses, s, len(part)) == part
    cat = b"".join(streams)
    rec = {
        "chunk_len": chunk_len,
        "n": len(syms),
        "lens": [len(s) for s in streams],
        "total_bytes": len(cat),
        "sha256": hashlib.sha256(cat).hexdigest(),
        "info_bits": info_bits(masses, syms),
    }
    if keep_bytes:
        rec["hex"] = cat.hex()
    return rec


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def small_cases():
    """Hand-picked tables that exercise the edge cases the reference tests use:
    zero masses (codec.rs:648), Bernoulli(2,10)/(0,10)/(10,10) (codec.rs:650-652),
    tiny and power-of-two norms, single-symbol chunks and ragged last chunks."""
    cases = []

    def add(name, masses, syms, chunk_len):
        cases.append({"name": name, "masses": masses, "syms": syms,
                      **record(masses, syms, chunk_len, keep_bytes=True)})

    add("dists_categorical", [0, 1, 2, 3, 0, 0, 1, 0], [1, 2, 3, 6, 3, 3, 2, 1, 6, 6, 3], 4)
    add("bernoulli_2_10", [8, 2], [0, 1, 1, 0, 0, 0, 1, 0, 1, 1, 1, 1, 0], 5)
    add("bernoulli_0_10", [10, 0], [0] * 17, 17)
    add("bernoulli_10_10", [0, 10], [1] * 9, 2)
    add("pow2_norm", [1 << 10, 1 << 12, 3 << 12, 1 << 10], [(i * 7) % 4 for i in range(300)], 64)
    add("single_symbol_chunks", [5, 9, 1, 300000], [3, 2, 1, 0, 3, 3, 2], 1)
    masses = [1 + splitmix64(0x5EED ^ s) % (1 << 20) for s in range(256)]
    _, norm = cumulative(masses)
    cums, _ = cumulative(masses)
    syms = []
    for i in range(5000):
        r = splitmix64((1 << 48) ^ i)
        cf = (r * norm) >> 64
        lo, hi = 0, len(cums)
        while lo < hi:
            mid = (lo + hi) // 2
            if cums[mid] <= cf:
                lo = mid + 1
            else:
                hi = mid
        syms.append(lo - 1)
    add("c3_table_first5000", masses, syms, 1024)
    return cases


def read_multiset(size):
    with open(os.path.join(REF, "multiset-data", f"{size}.txt")) as f:
        vals = [int(s) for s in f.read().split(", ")]
    assert len(vals) == size
    return vals


def main():
    if not os.path.isdir(REF):
        sys.exit("make_golden.py needs /root/reference (build container only)")
    src = open(os.path.join(REF, "src", "multiset.rs")).read()
    m = re.search(r"let probs = vec!\[([^\]]*)\];", src)
    probs = [float(s) for s in m.group(1).split(",")]
    assert len(probs) == 1024
    masses = [max(1, int(p * float(1 << 28))) for p in probs]
    with open(os.path.join(HERE, "masses_multiset.json"), "w") as f:
        json.dump({"source": "src/multiset.rs:158,169-170 (max(1, floor(p*2^28)))",
                   "norm": sum(masses), "masses": masses}, f)

    out = {"table": "masses_multiset.json", "init": "Message::zeros()", "vectors": {}}
    for size in (1000, 10000, 100000):
        shutil.copyfile(os.path.join(REF, "multiset-data", f"{size}.txt"),
                        os.path.join(HERE, f"multiset_{size}.txt"))
        syms = read_multiset(size)
        recs = {"single_chunk": record(masses, syms, size, keep_bytes=size <= 10000)}
        c2 = -(-size // 64)  # ceil(n / 64): SURVEY.md §8d config C2
        recs["chunks64"] = record(masses, syms, c2, keep_bytes=size <= 10000)
        out["vectors"][str(size)] = recs
        print(size, recs["single_chunk"]["total_bytes"], recs["chunks64"]["total_bytes"],
              round(recs["single_chunk"]["info_bits"], 1))
    with open(os.path.join(HERE, "golden_multiset.json"), "w") as f:
        json.dump(out, f)
    with open(os.path.join(HERE, "golden_small.json"), "w") as f:
        json.dump({"init": "Message::zeros()", "cases": small_cases()}, f)


if __name__ == "__main__":
    main()
