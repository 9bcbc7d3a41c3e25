"""CPU tests of the shipped library's host side (include/ans_capi.h sections 1-3).

The C ABI must load and export every symbol the header declares; the host Message /
Codec mirror must be byte-identical with the oracle and pass the reference's own
property tests (src/ans.rs:47-74, src/codec.rs:646-661).  No GPU is touched here.
"""
import ctypes
import math
import os
import random
import re

import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            text = open(os.path.join(inc, fn)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            names |= set(re.findall(r"\b(ans_\w+)\s*\(", text))
    return names


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(A.LIB_PATH)
    declared = _header_functions()
    assert len(declared) >= 35
    for name in sorted(declared):
        assert hasattr(L, name), f"{name} declared in include/ but not exported"
    assert declared == set(A.SIGNATURES), "Python binding out of sync with the header"
    assert A.lib().ans_abi_version() == 1


def test_no_gpu_here_fails_loudly():
    if A.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(A.AnsError) as e:
        A.Gpu(0)
    assert e.value.code == A.ANS_E_DEVICE


def test_gpu_entry_allocation_failure_is_a_status():
    """no exception crosses the ABI.  ans_gpu_graphs_decode sizes a std::vector by
    num_graphs before any device call; 2^62 entries exceed std::vector's max_size, so it throws
    std::length_error -- the entry's function-try-block returns ANS_E_ALLOC instead of aborting
    the (ctypes) caller.  No GPU and no real handle is needed to reach it."""
    L = A.lib()
    dummy = ctypes.create_string_buffer(64)  # never dereferenced before the throw
    nn = np.zeros(4, np.uint32)
    offs, lens, eo = np.zeros(4, np.uint64), np.zeros(4, np.uint64), np.zeros(4, np.uint64)
    rc = L.ans_gpu_graphs_decode(ctypes.cast(dummy, ctypes.c_void_p), A.ANS_NO_TABLE, A.ANS_NO_TABLE, 0, 0, 0, 1 << 62,
                                 A._np_ptr(nn), None, 0, A._np_ptr(offs), A._np_ptr(lens), A.GEN_ZEROS, 0, None, None,
                                 None, 0, A._np_ptr(eo))
    assert rc == A.ANS_E_ALLOC


def test_every_gpu_entry_is_exception_guarded():
    """Every extern "C" definition of the HIP units is a function-try-block ending in ANS_CATCH
    (shuffle-coding_amd/csrc/ans_ctx.hpp), except one-line bodies that cannot throw."""
    csrc = os.path.join(ROOT, "shuffle-coding_amd", "csrc")
    unguarded = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith(".hip"):
            continue
        text = open(os.path.join(csrc, fn)).read()
        n_defs = 0
        for block in re.findall(r'^extern "C" \{\n(.*?)^\}  // extern "C"', text, flags=re.S | re.M):
            lines = block.split("\n")
            for i, line in enumerate(lines):
                m = re.match(r"(?:int|void|uint64_t) ((?:ans|dev)_\w+)\(", line)
                if not m or line.rstrip().endswith("}"):  # (a declaration-free one-liner)
                    continue
                n_defs += 1
                j = next(k for k in range(i, len(lines)) if lines[k].rstrip().endswith("{"))
                end = next(k for k in range(j + 1, len(lines)) if lines[k].startswith("}"))
                if not (lines[j].rstrip().endswith(") try {") and lines[end].startswith("} ANS_CATCH")):
                    unguarded.append(f"{fn}:{m.group(1)}")
        if fn in ("ans_kernels.hip", "ans_codecs.hip", "ans_graph.hip"):
            assert n_defs >= 9, fn
    assert not unguarded, unguarded


def test_multiset_single_message_matches_golden(multiset_masses, multiset_vectors, golden_multiset):
    cat = A.Categorical(multiset_masses)
    for size, syms in multiset_vectors.items():
        rec = golden_multiset["vectors"][str(size)]["single_chunk"]
        m = A.Message.zeros()
        A.IID(cat, size).push(m, syms)
        data = m.flatten()
        assert len(data) == rec["total_bytes"]
        if "hex" in rec:
            assert data.hex() == rec["hex"]
        back = A.IID(cat, size).pop(A.Message.unflatten(data))
        assert back == syms.tolist()


def test_random_op_sequences_match_oracle():
    rng = random.Random(1234)
    tables = [[0, 1, 2, 3, 0, 0, 1, 0], [8, 2], [1] * 7, [rng.randrange(1, 1 << 20) for _ in range(300)],
              [1 << 40, 3, 1 << 30], [rng.randrange(0, 5) for _ in range(50)] + [1]]
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 7), (A.GEN_RANDOM, 0)]:
        pm = A.Message._new(kind, seed)
        om = orc.lib().orc_msg_new(kind, seed)
        om = orc.Message(om)
        assert pm.head == om.head
        pcats = [A.Categorical(t) for t in tables]
        ocats = [orc.Categorical(t) for t in tables]
        for _ in range(3000):
            op = rng.randrange(5)
            if op < 2:
                k = rng.randrange(len(tables))
                nz = [i for i, v in enumerate(tables[k]) if v]
                x = rng.choice(nz)
                pcats[k].push(pm, x)
                assert ocats[k].push(om, x) == 0
            elif op < 4:
                k = rng.randrange(len(tables))
                assert pcats[k].pop(pm) == ocats[k].pop(om)
            else:
                size = rng.choice([2, 3, 1 << 28, (1 << 46) - 1, 1000003])
                if rng.random() < 0.5:
                    x = rng.randrange(size)
                    A.Uniform(size).push(pm, x)
                    assert orc.uniform_push(om, size, x) == 0
                else:
                    assert A.Uniform(size).pop(pm) == orc.uniform_pop(om, size)
            assert pm.head == om.head
        assert pm.flatten() == om.flatten()
        assert pm.bits() == om.bits()
        assert math.isclose(pm.virtual_bits(), om.virtual_bits(), rel_tol=0, abs_tol=1e-9)


def test_reference_property_dists():
    # src/codec.rs:646-656 on the shipped host coder
    def check(codec, h):
        am = codec.test_on_samples(1000)
        assert abs(sum(am) / len(am) - h) / max(abs(h), 1) < 0.02

    c = A.Categorical([0, 1, 2, 3, 0, 0, 1, 0])
    check(c, c.entropy())
    for mass, norm in [(2, 10), (0, 10), (10, 10)]:
        b = A.Bernoulli(mass, norm)
        check(b, b.categorical.entropy())
    A.Uniform(1 << 28).test_on_samples(1000)
    A.IID(A.Uniform(1 << 28), 2).test_on_samples(300)
    A.Independent([A.Uniform(1 << 28)] * 2).test_on_samples(300)


class _ShuffledWithin(A.Distribution):
    """A Distribution whose cdf(x, i) is NOT cum[x] + i (like PlainOrbitCodec,
    src/recursive/plain_orbit.rs:33-49): exercises the two-phase scalar ABI."""

    def __init__(self, masses):
        self.masses = masses
        self.cums = [sum(masses[:k]) for k in range(len(masses))]

    def norm(self):
        return sum(self.masses)

    def pmf(self, x):
        return self.masses[x]

    def cdf(self, x, i):
        return self.cums[x] + (self.masses[x] - 1 - i)

    def icdf(self, cf):
        x = max(k for k in range(len(self.cums)) if self.cums[k] <= cf and self.masses[k])
        return x, self.masses[x] - 1 - (cf - self.cums[x])


def test_two_phase_scalar_abi_with_custom_cdf():
    d = _ShuffledWithin([5, 1, 0, 9, 300, 2])
    d.test_on_samples(300)
    IIDd = A.IID(d, 40)
    for seed in range(20):
        IIDd.test(IIDd.sample(seed), A.Message.zeros())


def test_error_codes_mirror_reference_panics():
    c = A.Categorical([3, 0, 2])
    with pytest.raises(A.AnsError) as e:
        c.push(A.Message.zeros(), 1)  # src/ans.rs:98 assert_ne!(p, 0)
    assert e.value.code == A.ANS_E_ZERO_MASS
    with pytest.raises(A.AnsError) as e:
        c.push(A.Message.zeros(), 3)  # src/codec.rs:63 index out of bounds
    assert e.value.code == A.ANS_E_SYMBOL
    m = A.Message.empty()
    with pytest.raises(A.AnsError) as e:
        for _ in range(50):
            c.pop(m)  # src/ans.rs:144
    assert e.value.code == A.ANS_E_EXHAUSTED
    with pytest.raises(AssertionError):
        A.Uniform(A.MAX_SIZE + 1)  # src/codec.rs:35
    with pytest.raises(AssertionError):
        A.IID(c, 3).push(A.Message.zeros(), np.array([0, 2], np.uint32))  # src/codec.rs:416


def test_message_equality_canonicalises():
    # src/ans.rs:302-310: equal after renorm to MAX_MIN_HEAD and tail normalisation
    z = A.Message.zeros()
    u = A.Message.unflatten(z.flatten())
    assert z == u
    r = A.Message.random(3)
    assert r == r.reflatten()
    assert r != A.Message.random(4)
    assert A.Message.zeros() != A.Message.empty()


def test_truncated_benford_log_uniform():
    # src/codec.rs:663-669: LogUniform::new(8) passes Codec::test for x < 255 from Message::random(0);
    # bytes equal the oracle's composition of Uniform pushes (src/codec.rs:569-577)
    c = A.LogUniform(8)
    for i in range(255):
        c.test(i, A.Message.random(0))
    m = A.Message.zeros()
    om = orc.Message.zeros()
    xs = [0, 1, 2, 3, 7, 8, 200, 254, 100, 5]
    for x in xs:
        c.push(m, x)
        b = x.bit_length()
        if b:
            assert orc.uniform_push(om, 1 << (b - 1), x & ~(1 << (b - 1))) == 0
        assert orc.uniform_push(om, 9, b) == 0
    assert m.flatten() == om.flatten()
    assert [c.pop(m) for _ in xs] == xs[::-1]
    big = A.LogUniform.max()  # MaxBenfordIID's item: 47-bit values
    m = A.Message.zeros()
    for x in [(1 << 46) + 12345, 1, 0, (1 << 40) - 1]:
        big.push(m, x)
        assert big.pop(m) == x
