"""The LDS fast kernels outside 2^16 <= norm <= 2^31 (ans_fast.hpp kNormSmall / kNormBig,
DESIGN.md §4b), bit-exact against the oracle.

The reference builds its dataset-level tables from counts: the edge Bernoulli
`Bernoulli::new(total_edges, total_possible_edges)` and the node / edge label Categoricals
(src/benchmark.rs:549-578), `Bernoulli::new(1, 2)` for the loops flag (src/param_codec.rs:273).
Ordinary datasets give norms below 2^16; very large ones can pass 2^31.  Those tables used to
take the one-lane generic kernels; every table here must now report the LDS fast paths (or, above
256 symbols, the large-alphabet ones) and code every chunk to the oracle's bytes (fixed chunks,
ragged chunks through the staged kernels, variable-length chunks, Message::random initial
messages).
"""
import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    return A.Gpu(0)


def _spread(rng, nsym, norm):
    """nsym positive masses summing exactly to norm (distinct cut points)."""
    cuts = np.zeros(0, np.int64)
    while len(cuts) < nsym - 1:
        cuts = np.unique(np.concatenate([cuts, rng.integers(1, norm, 2 * nsym, dtype=np.int64)]))
    cuts = np.sort(rng.permutation(cuts)[:nsym - 1])
    return np.diff(np.concatenate([[0], cuts, [norm]])).astype(np.uint64)


def _dataset_bernoulli(rng, num_graphs=188, mean_nodes=18):
    """DatasetStats::unlabelled's edge Bernoulli (src/benchmark.rs:550-557) for a MUTAG-shaped
    set of undirected graphs: [possible - edges, edges] with norm = sum of n (n - 1) / 2."""
    nodes = np.maximum(2, rng.normal(mean_nodes, 4, num_graphs).astype(np.int64))
    possible = int((nodes * (nodes - 1) // 2).sum())
    edges = int((nodes * 1.1).astype(np.int64).sum())
    return np.asarray([possible - edges, edges], np.uint64)


TABLES = {
    # norm < 2^16 (kNormSmall)
    "bernoulli_1_2": lambda r: np.asarray([1, 1], np.uint64),  # src/param_codec.rs:273; norm 2 = 2^1
    "dataset_edges": lambda r: _dataset_bernoulli(r),          # norm ~3e4
    "node_labels": lambda r: np.asarray([2395, 345, 593, 0, 23, 12, 2], np.uint64),  # counts, one absent label
    "norm_3": lambda r: np.asarray([1, 2], np.uint64),
    "norm_255": lambda r: _spread(r, 40, 255),                 # 24-bit high-word product off (norm <= 256)
    "norm_256_ones": lambda r: np.ones(256, np.uint64),       # L = 2^56, every mass 1
    "norm_257": lambda r: _spread(r, 100, 257),               # ... on again
    "norm_2^16-1": lambda r: _spread(r, 256, (1 << 16) - 1),
    "c3_small": lambda r: A.c3_small_masses(),                 # bench.py --config c3s, norm 32,749
    "skewed_small": lambda r: np.concatenate([[60000], np.ones(200, np.int64)]).astype(np.uint64),
    # 2^31 < norm < 2^32 (kNormBig)
    "norm_2^31+1": lambda r: _spread(r, 256, (1 << 31) + 1),
    "c3_big": lambda r: A.c3_big_masses(),                     # bench.py --config c3b, norm 2^32 - 5
    "mass_above_2^31": lambda r: np.concatenate([[(1 << 31) + 12345, 1, 77, 1 << 30],
                                                 r.integers(1, 1 << 20, 60)]).astype(np.uint64),
    "norm_2^32-1_two": lambda r: np.asarray([(1 << 32) - 2, 1], np.uint64),
    "kmax4_big": lambda r: np.concatenate([[1, 1, 2], _spread(r, 200, (1 << 32) - 100)]).astype(np.uint64),
}
SMALL = ["bernoulli_1_2", "dataset_edges", "node_labels", "norm_3", "norm_255", "norm_256_ones", "norm_257",
         "norm_2^16-1", "c3_small", "skewed_small"]
BIG = ["norm_2^31+1", "c3_big", "mass_above_2^31", "norm_2^32-1_two", "kmax4_big"]


def _table(name):
    masses = TABLES[name](np.random.default_rng(sum(map(ord, name))))
    norm = int(masses.sum())
    assert norm < (1 << 16) if name in SMALL else (1 << 31) < norm < (1 << 32)
    return masses


def _symbols(masses, n, seed):
    """Half iid from the table, half uniform over its symbols (so rare rows are coded often)."""
    rng = np.random.default_rng(seed)
    nz = np.flatnonzero(masses)
    syms = orc.gen_iid(masses, seed, 0, n)
    mask = rng.random(n) < 0.5
    syms[mask] = rng.choice(nz, size=int(mask.sum()))
    return syms.astype(np.uint32)


def _roundtrip(gt, masses, syms, chunk_len, dtype, **kw):
    s = syms.astype(dtype)
    data, offsets, lens = gt.encode_chunks(s, chunk_len, **kw)
    okw = {} if not kw else {"kind": orc.RANDOM, "seed": kw["seed"]}
    od, oo, ol = orc.encode_chunks(masses, syms, chunk_len, **okw)
    assert np.array_equal(lens, ol)
    assert np.array_equal(offsets, oo)
    assert data.tobytes() == od.tobytes()
    back = gt.decode_chunks(data, offsets, lens, len(s), chunk_len, dtype, **kw)
    assert np.array_equal(back, s)


@pytest.mark.parametrize("name", SMALL + BIG)
def test_norm_range_tables_take_the_fast_kernels(gpu, name):
    masses = _table(name)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    p = gt.paths()
    assert p & A.ANS_PATH_ENC_LDS and p & A.ANS_PATH_DEC_LDS, hex(p)
    n = 300 * 4096 + 77  # full chunks on the fast kernels, the ragged last one generic
    syms = _symbols(masses, n, 3)
    for dtype in (np.uint8, np.uint16, np.uint32):
        _roundtrip(gt, masses, syms, 4096, dtype)


@pytest.mark.parametrize("name", ["dataset_edges", "node_labels", "c3_small", "norm_255", "c3_big", "mass_above_2^31"])
@pytest.mark.parametrize("chunk_len", [1563, 64])
def test_norm_range_staged_chunks(gpu, name, chunk_len):
    """Chunk lengths off the 128-B groups: the staged kVar kernels."""
    masses = _table(name)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    syms = _symbols(masses, 700 * chunk_len + 11, 5)
    _roundtrip(gt, masses, syms, chunk_len, np.uint8)


@pytest.mark.parametrize("name", ["bernoulli_1_2", "dataset_edges", "c3_small", "c3_big"])
def test_norm_range_random_messages(gpu, name):
    """Message::random(seed + c) initial messages (src/ans.rs:285-290)."""
    masses = _table(name)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    syms = _symbols(masses, 520 * 4096, 7)
    _roundtrip(gt, masses, syms, 4096, np.uint8, gen_kind=A.GEN_RANDOM, seed=999)


@pytest.mark.parametrize("name", ["dataset_edges", "node_labels", "c3_small", "c3_big"])
def test_norm_range_var_chunks(gpu, name):
    """One chunk per graph (variable lengths, empty ones included): each stream is the reference
    message of its slice alone."""
    masses = _table(name)
    rng = np.random.default_rng(13)
    sizes = np.concatenate([[0, 1, 0, 7], rng.integers(0, 3000, 600), [20000, 0]]).astype(np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    syms = _symbols(masses, int(starts[-1]), 11)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    data, offsets, lens = gt.encode_var_chunks(syms.astype(np.uint8), starts)
    for c in range(len(sizes)):
        a, b = int(starts[c]), int(starts[c + 1])
        od, _, _ = orc.encode_chunks(masses, syms[a:b], max(b - a, 1))
        want = od.tobytes() if b > a else bytes(orc.Message.zeros().flatten())
        assert data[int(offsets[c]):int(offsets[c] + lens[c])].tobytes() == want, c
    back = gt.decode_var_chunks(data, offsets, lens, starts, np.uint8)
    assert np.array_equal(back, syms.astype(np.uint8))


@pytest.mark.parametrize("name", ["c3_small", "c3_big"])
def test_norm_range_whole_gib(gpu, name):
    """bench.py's c3s / c3b workloads (2^30 u8 symbols, chunk 4096) on the device, byte-checked
    like C3 itself (test_gpu_parity._device_roundtrip): every one of the 262,144 chunks' lengths,
    and the bytes of the whole dense container as a sha256 per slice of chunks against the
    oracle's streams of the same counter-based symbols; the round trip is lossless from the slots
    and from the dense container."""
    from test_gpu_parity import _device_roundtrip
    total = _device_roundtrip(gpu, _table(name), 1 << 30, 4096, 1, 1)
    assert 0.9 < total / (1 << 30) < 1.0


# ---- more than 256 symbols outside [2^16, 2^31]: the large-alphabet kernels' kNormSmall /
# kNormBig division (ans_fast.hpp k_encode with global rows and k_decode_g, ans_wide.hpp
# k_encode_w / k_decode_w with kNR)
def _label_counts(rng, nsym, total):
    """A count-built label Categorical (DatasetStats::dist, src/benchmark.rs:576-578): Zipf-like
    counts over nsym labels, some labels absent (zero mass), summing to about `total`."""
    w = 1.0 / np.arange(1, nsym + 1) ** 0.9
    c = np.floor(w / w.sum() * total).astype(np.int64)
    c[rng.choice(nsym, size=nsym // 10, replace=False)] = 0
    c[0] = max(c[0], 1)
    return c.astype(np.uint64)


WIDE = {
    # kNormSmall
    "labels_4096_norm_6e4": lambda r: _label_counts(r, 4096, 60000),
    "wide_300_norm_1000": lambda r: _spread(r, 300, 1000),
    "wide_65536_ones": lambda r: np.ones(65535, np.uint64),  # norm 2^16 - 1, every mass 1
    # kNormBig
    "wide_1000_norm_2^32-5": lambda r: _spread(r, 1000, (1 << 32) - 5),
    "wide_65536_mass_above_2^31": lambda r: np.concatenate([[(1 << 31) + 999], r.integers(1, 1 << 14, 65535)]).astype(
        np.uint64),
}


def _wide(name):
    masses = WIDE[name](np.random.default_rng(sum(map(ord, name))))
    norm = int(masses.sum())
    assert len(masses) > 256 and (norm < (1 << 16) or (1 << 31) < norm < (1 << 32)), norm
    return masses


@pytest.mark.parametrize("name", sorted(WIDE))
def test_wide_norm_range_tables_take_the_fast_kernels(gpu, name):
    masses = _wide(name)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    p = gt.paths()
    assert p & (A.ANS_PATH_ENC_GLOBAL | A.ANS_PATH_ENC_WIDE), hex(p)
    assert p & (A.ANS_PATH_DEC_GLOBAL | A.ANS_PATH_DEC_WIDE), hex(p)
    n = 300 * 4096 + 77  # full chunks on the fast kernels, the ragged last one generic
    syms = _symbols(masses, n, 3)
    for dtype in (np.uint16, np.uint32):
        _roundtrip(gt, masses, syms, 4096, dtype)
    _roundtrip(gt, masses, syms[:200 * 1563 + 5], 1563, np.uint16)  # staged (ragged) chunks
    _roundtrip(gt, masses, syms[:520 * 4096], 4096, np.uint16, gen_kind=A.GEN_RANDOM, seed=4)


@pytest.mark.parametrize("name", ["labels_4096_norm_6e4", "wide_65536_mass_above_2^31"])
def test_wide_norm_range_var_chunks(gpu, name):
    masses = _wide(name)
    rng = np.random.default_rng(17)
    sizes = np.concatenate([[0, 1, 7], rng.integers(0, 2500, 300), [9000, 0]]).astype(np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    syms = _symbols(masses, int(starts[-1]), 19).astype(np.uint16)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    data, offsets, lens = gt.encode_var_chunks(syms, starts)
    for c in range(len(sizes)):
        a, b = int(starts[c]), int(starts[c + 1])
        od, _, _ = orc.encode_chunks(masses, syms[a:b].astype(np.uint32), max(b - a, 1))
        want = od.tobytes() if b > a else bytes(orc.Message.zeros().flatten())
        assert data[int(offsets[c]):int(offsets[c] + lens[c])].tobytes() == want, c
    back = gt.decode_var_chunks(data, offsets, lens, starts, np.uint16)
    assert np.array_equal(back, syms)
