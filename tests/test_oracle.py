"""Pins the C oracle (oracle/ans_oracle.c) before anything is checked against it.

* against the committed golden vectors (tests/golden/, made by an independent pure-Python
  restatement from the reference's own fixtures multiset-data/*.txt and table rule
  src/multiset.rs:158,169-170);
* against the reference's own property tests, re-run on the oracle:
  Codec::test / test_invertibility (src/ans.rs:47-68) and `dists` (src/codec.rs:646-661).
"""
import hashlib
import math

import numpy as np
import pytest

from oracle import oracle as orc


def test_multiset_table_rule(multiset_masses):
    # src/multiset.rs:169-170: masses max(1, floor(p * 2^28)) -> norm 268,434,941
    assert len(multiset_masses) == 1024
    assert int(multiset_masses.sum()) == 268_434_941
    assert int(multiset_masses.min()) == 407 and int(multiset_masses.max()) == 550_552


@pytest.mark.parametrize("size", [1000, 10000, 100000])
@pytest.mark.parametrize("layout", ["single_chunk", "chunks64"])
def test_oracle_matches_golden_multiset(size, layout, multiset_masses, multiset_vectors, golden_multiset):
    rec = golden_multiset["vectors"][str(size)][layout]
    syms = multiset_vectors[size]
    data, offsets, lens = orc.encode_chunks(multiset_masses, syms, rec["chunk_len"])
    assert [int(x) for x in lens] == rec["lens"]
    assert hashlib.sha256(data.tobytes()).hexdigest() == rec["sha256"]
    if "hex" in rec:
        assert data.tobytes().hex() == rec["hex"]
    back = orc.decode_chunks(multiset_masses, data, offsets, lens, len(syms), rec["chunk_len"])
    assert np.array_equal(back, syms)


def test_oracle_matches_golden_small(golden_small):
    for case in golden_small:
        data, offsets, lens = orc.encode_chunks(case["masses"], case["syms"], case["chunk_len"])
        assert data.tobytes().hex() == case["hex"], case["name"]
        assert [int(x) for x in lens] == case["lens"], case["name"]
        back = orc.decode_chunks(case["masses"], data, offsets, lens, len(case["syms"]), case["chunk_len"])
        assert back.tolist() == case["syms"], case["name"]


def test_amortized_bits_equal_information_content(multiset_masses, multiset_vectors, golden_multiset):
    # Codec::test: amortized bits == bits(x) within 1e-5 (src/ans.rs:62-68, 325-327)
    cat = orc.Categorical(multiset_masses)
    for size, syms in multiset_vectors.items():
        init = orc.Message.zeros()
        m = init.clone()
        assert cat.push_iid(m, syms) == 0
        amortized = m.virtual_bits() - init.virtual_bits()
        expected = golden_multiset["vectors"][str(size)]["single_chunk"]["info_bits"]
        assert abs(amortized - expected) / max(abs(expected), 1) < 1e-5
        assert m.bits() >= amortized
        assert m.bits() == 8 * golden_multiset["vectors"][str(size)]["single_chunk"]["total_bytes"]


# ---------------------------------------------------------------- reference property tests
class _OracleCat:
    def __init__(self, masses):
        self.c = orc.Categorical(masses)
        self.masses = [int(x) for x in masses]
        self.norm = sum(self.masses)

    def push(self, m, x):
        assert self.c.push(m, x) == 0

    def pop(self, m):
        return self.c.pop(m)

    def bits(self, x):
        return math.log2(self.norm) - math.log2(self.masses[x])


class _OracleUniform:
    def __init__(self, size):
        self.size = size

    def push(self, m, x):
        assert orc.uniform_push(m, self.size, x) == 0

    def pop(self, m):
        return orc.uniform_pop(m, self.size)

    def bits(self, x):
        return math.log2(self.size)


class _OracleIID:
    def __init__(self, item, n):
        self.item, self.n = item, n

    def push(self, m, xs):
        for x in reversed(xs):
            self.item.push(m, x)

    def pop(self, m):
        return [self.item.pop(m) for _ in range(self.n)]

    def bits(self, xs):
        return sum(self.item.bits(x) for x in xs)


def _test(codec, x, initial):
    """Codec::test (src/ans.rs:47-68) on the oracle."""
    m = initial.clone()
    codec.push(m, x)
    bits = m.bits()
    amortized = m.virtual_bits() - initial.virtual_bits()
    assert bits >= amortized
    assert codec.pop(m) == x
    assert initial == m
    assert initial == m.reflatten()
    expected = codec.bits(x)
    assert abs(amortized - expected) / max(abs(expected), 1) < 1e-5
    return amortized


def _test_on_samples(codec, num):
    """Codec::test_on_samples (src/ans.rs:72-74): sample(seed) pops from Message::random(seed)."""
    out = []
    for seed in range(num):
        x = codec.pop(orc.Message.random(seed))
        out.append(_test(codec, x, orc.Message.random(seed)))
    return out


def _entropy(masses):
    n = sum(masses)
    return -sum(m / n * math.log2(m / n) for m in masses if m)


@pytest.mark.parametrize("masses", [[0, 1, 2, 3, 0, 0, 1, 0], [8, 2], [10, 0], [0, 10]])
def test_dists_categorical_and_bernoulli(masses):
    # src/codec.rs:646-661: mean amortized bits within 2 % of the entropy
    amortized = _test_on_samples(_OracleCat(masses), 1000)
    h = _entropy(masses)
    assert abs(sum(amortized) / len(amortized) - h) / max(abs(h), 1) < 0.02


def test_dists_uniform_and_iid():
    # src/codec.rs:653-655
    _test_on_samples(_OracleUniform(1 << 28), 1000)
    iid = _OracleIID(_OracleUniform(1 << 28), 2)
    for seed in range(200):
        x = iid.pop(orc.Message.random(seed))
        _test(iid, x, orc.Message.random(seed))


def test_zeros_and_empty_generators():
    m = orc.Message.empty()
    cat = orc.Categorical([1, 2, 3])
    with pytest.raises(RuntimeError):
        for _ in range(100):  # Empty generator panics once the head underflows (src/ans.rs:144)
            cat.pop(m)
    z = orc.Message.zeros()
    for _ in range(100):
        cat.pop(z)
    assert z.num_generated > 0


def test_gen_iid_matches_python_splitmix():
    masses = [3, 0, 5, 1 << 20, 7]
    cums = np.concatenate([[0], np.cumsum(masses)[:-1]])
    norm = sum(masses)
    ref = []
    for i in range(500):
        r = orc.splitmix64((9 << 48) ^ (100 + i))
        cf = (r * norm) >> 64
        ref.append(int(np.searchsorted(cums, cf, side="right")) - 1)
    assert orc.gen_iid(masses, 9, 100, 500).tolist() == ref


def test_random_initial_message_containers(multiset_masses, multiset_vectors):
    """Chunks begun as Message::random(seed + c) (the reference harness' initial message,
    src/multiset.rs:174): the oracle's container equals the host coder's IID push on
    Message::random, and decoding with the tail's generator state kept (src/ans.rs:57) returns
    every chunk to its initial message (src/ans.rs:56)."""
    import ans_amd as A
    syms = multiset_vectors[10000]
    cat = A.Categorical(multiset_masses)
    d, o, ln = orc.encode_chunks(multiset_masses, syms, len(syms), kind=orc.RANDOM, seed=0)
    m = A.Message.random(0)
    A.IID(cat, len(syms)).push(m, syms)
    assert m.flatten() == d.tobytes()  # the reference harness' single message
    for chunk_len, seed in [(len(syms), 0), (157, 5), (1, 11)]:
        d, o, ln = orc.encode_chunks(multiset_masses, syms, chunk_len, kind=orc.RANDOM, seed=seed)
        back = orc.decode_chunks(multiset_masses, d, o, ln, len(syms), chunk_len, kind=orc.RANDOM, seed=seed)
        assert np.array_equal(back, syms)
        for c in (0, len(ln) - 1):  # chunk c is the host coder's message from Message::random(seed + c)
            a, b = c * chunk_len, min(len(syms), (c + 1) * chunk_len)
            mm = A.Message.random(seed + c)
            A.IID(cat, b - a).push(mm, syms[a:b])
            assert mm.flatten() == d[int(o[c]):int(o[c]) + int(ln[c])].tobytes()
        with pytest.raises(RuntimeError):  # the wrong seed does not return to the initial message
            orc.decode_chunks(multiset_masses, d, o, ln, len(syms), chunk_len, kind=orc.RANDOM, seed=seed + 1)
