"""The graph models' bulk-IID caller: DenseSetIID<EdgeIndex, AllEdgeIndices> with
IID<Bernoulli> (ErdosRenyi, src/graph_codec.rs:104-205).

CPU: the host mirror (ans_amd.AllEdgeIndices / ErdosRenyi on one Message) against the oracle's
literal restatement of the alphabet order (src/graph_codec.rs:187-199) and its IID coder.
GPU (`gpu` marker): the device edge <-> dense kernels and the chunked Bernoulli coding through
the C ABI (ans_gpu_dense_set_encode / _decode), bit-exact per chunk against the oracle.
"""
import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

NORM = 1 << 28  # plain_erdos_renyi's Bernoulli norm (src/graph_codec.rs:399-401)


def _er_masses(p):
    mass = int(p * NORM)  # (p * norm as f64) as usize
    return [NORM - mass, mass], mass


def _random_graph(rng, n, p, directed, loops):
    alpha = orc.all_edge_indices(n, directed, loops) if n <= 400 else None
    if alpha is not None:
        keep = rng.random(len(alpha)) < p
        return np.asarray([e for e, k in zip(alpha, keep) if k], dtype=np.uint32).reshape(-1, 2)
    m = rng.binomial(n * (n - 1) // 2, p)
    i = rng.integers(0, n, size=2 * m)
    j = rng.integers(0, n, size=2 * m)
    a, b = np.minimum(i, j), np.maximum(i, j)
    e = np.unique(np.stack([a, b], 1)[a != b], axis=0)[:m]
    if directed:
        flip = rng.random(len(e)) < 0.5
        e[flip] = e[flip][:, ::-1]
    return e.astype(np.uint32)


def _alphabet_sorted(edges, n, directed, loops):
    s = orc.edge_slots(edges, n, directed, loops)
    u, idx = np.unique(s, return_index=True)
    return np.asarray(edges, dtype=np.uint32).reshape(-1, 2)[idx]


# ---------------------------------------------------------------- host mirror (CPU)
@pytest.mark.parametrize("n", [0, 1, 2, 7])
@pytest.mark.parametrize("directed", [False, True])
@pytest.mark.parametrize("loops", [False, True])
def test_alphabet_order_matches_reference(n, directed, loops):
    ref = orc.all_edge_indices(n, directed, loops)
    alpha = A.AllEdgeIndices(n, directed, loops)
    assert list(alpha) == ref
    assert len(alpha) == len(ref)
    if ref:
        assert np.array_equal(orc.edge_slots(ref, n, directed, loops), np.arange(len(ref)))


@pytest.mark.parametrize("directed,loops", [(False, False), (True, False), (False, True), (True, True)])
def test_erdos_renyi_host_message_bit_exact(directed, loops):
    rng = np.random.default_rng(1 + 2 * directed + loops)
    n, p = 23, 0.2
    masses, mass = _er_masses(p)
    edges = _random_graph(rng, n, p, directed, loops)
    er = A.ErdosRenyi(A.Bernoulli(mass, NORM), n, directed, loops)
    m = A.Message.zeros()
    er.push(m, [tuple(map(int, e)) for e in edges])
    om = orc.Message.zeros()
    assert orc.Categorical(masses).push_iid(om, orc.dense_set(edges, n, directed, loops)) == 0
    assert m.flatten() == om.flatten()
    back = er.pop(m)
    assert back == [tuple(map(int, e)) for e in _alphabet_sorted(edges, n, directed, loops)]
    assert m == A.Message.zeros()
    # Codec::test semantics (src/ans.rs:47-68) on the same graph
    er.test([tuple(map(int, e)) for e in _alphabet_sorted(edges, n, directed, loops)], A.Message.zeros())


def test_dense_set_rejects_edges_outside_the_alphabet():
    er = A.ErdosRenyi(A.Bernoulli(1 << 20, NORM), 5, directed=False, loops=False)
    with pytest.raises(A.AnsError):
        er.push(A.Message.zeros(), [(3, 1)])  # undirected alphabet holds (1, 3) only
    with pytest.raises(A.AnsError):
        er.push(A.Message.zeros(), [(2, 2)])  # no loops


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("directed,loops", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("chunk_len", [4096, 1000])
def test_gpu_dense_set_bit_exact(directed, loops, chunk_len):
    rng = np.random.default_rng(7 + chunk_len + 2 * directed + loops)
    n, p = 300, 0.05
    masses, mass = _er_masses(p)
    edges = _random_graph(rng, n, p, directed, loops)
    gs = A.GpuDenseSet(A.Gpu(0), A.Bernoulli(mass, NORM), n, directed, loops)
    data, offsets, lens = gs.encode(edges, chunk_len)
    od, oo, ol = orc.encode_chunks(masses, orc.dense_set(edges, n, directed, loops), chunk_len)
    assert np.array_equal(lens, ol) and np.array_equal(offsets, oo)
    assert data.tobytes() == od.tobytes()
    back = gs.decode(data, offsets, lens, chunk_len)
    assert np.array_equal(back, _alphabet_sorted(edges, n, directed, loops))


@pytest.mark.gpu
def test_gpu_dense_set_large_undirected():
    """n = 20,000 (2e8 slots, 48,829 chunks of 4096): round trip, sampled chunks vs oracle."""
    rng = np.random.default_rng(3)
    n, p = 20_000, 1e-3
    masses, mass = _er_masses(p)
    edges = _random_graph(rng, n, p, False, False)
    gs = A.GpuDenseSet(A.Gpu(0), A.Bernoulli(mass, NORM), n)
    L = 4096
    data, offsets, lens = gs.encode(edges, L)
    back = gs.decode(data, offsets, lens, L)
    assert np.array_equal(back, _alphabet_sorted(edges, n, False, False))
    dense = orc.dense_set(edges, n, False, False)
    for j in sorted(set(rng.integers(0, len(lens), 16).tolist()) | {0, len(lens) - 1}):
        od, _, ol = orc.encode_chunks(masses, dense[j * L:(j + 1) * L], L)
        assert data[int(offsets[j]):int(offsets[j] + lens[j])].tobytes() == od.tobytes()


@pytest.mark.gpu
def test_gpu_dense_set_edge_cases():
    g = A.Gpu(0)
    masses, mass = _er_masses(0.3)
    gs = A.GpuDenseSet(g, A.Bernoulli(mass, NORM), 40)
    # outside the alphabet -> ANS_E_SYMBOL (the reference panics, src/graph_codec.rs:137)
    for bad in ([[5, 2]], [[4, 4]], [[1, 40]]):
        with pytest.raises(A.AnsError) as e:
            gs.encode(np.asarray(bad), 256)
        assert e.value.code == A.ANS_E_SYMBOL
    # duplicates collapse (the reference's HashSet), the empty graph, the complete graph
    full = np.asarray(orc.all_edge_indices(40, False, False), dtype=np.uint32)
    for edges in (np.zeros((0, 2), np.uint32), np.concatenate([full[:50], full[:50]]), full):
        data, offsets, lens = gs.encode(edges, 256)
        od, _, _ = orc.encode_chunks(masses, orc.dense_set(edges, 40, False, False), 256)
        assert data.tobytes() == od.tobytes()
        back = gs.decode(data, offsets, lens, 256, cap=3)  # too small: the second pass sizes it
        assert np.array_equal(back, _alphabet_sorted(edges, 40, False, False) if len(edges) else back[:0])
    # nodes = 0 and 1: empty alphabets
    for n in (0, 1):
        z = A.GpuDenseSet(g, A.Bernoulli(mass, NORM), n)
        data, offsets, lens = z.encode(np.zeros((0, 2), np.uint32), 64)
        assert len(data) == 0 and len(z.decode(data, offsets, lens, 64)) == 0


def _dataset_masses(nums, graphs, directed, loops, table):
    """The dataset's Bernoulli: plain_erdos_renyi's (norm 2^28, src/graph_codec.rs:399-401), or
    DatasetStats::unlabelled's Bernoulli::new(total_edges, total_possible_edges)
    (src/benchmark.rs:550-557), whose norm is below 2^16 for a set of small graphs."""
    if table == "er_2^28":
        return _er_masses(0.08)
    possible = sum(len(orc.all_edge_indices(n, directed, loops)) if n <= 400 else 0 for n in nums)
    edges = sum(len(e) for e in graphs)
    return [possible - edges, edges], edges


@pytest.mark.gpu
@pytest.mark.parametrize("directed,loops", [(False, False), (True, True)])
@pytest.mark.parametrize("table", ["er_2^28", "dataset_counts"])
def test_gpu_graph_dataset_bit_exact(directed, loops, table):
    """A dataset under one Bernoulli (GraphDatasetParamCodec + ErdosRenyiParamCodec,
    src/param_codec.rs:171-199,243-293): graph g's stream is the oracle's message of that graph's
    dense edge vector alone, and the host ErdosRenyi push of the graph; decoding returns every
    graph's edges in alphabet order.  dataset_counts (norm ~4e4 < 2^16) takes the LDS fast
    kernels' kNormSmall division (ans_fast.hpp)."""
    rng = np.random.default_rng(11 + directed)
    top = 60 if table == "er_2^28" else 40  # (a counts table of these graphs stays below 2^16)
    nums = [int(x) for x in rng.integers(0, top, 80)] + [0, 1, 2, 100 if directed else 150]
    p = 0.08
    graphs = [_random_graph(rng, n, p, directed, loops) for n in nums]
    masses, mass = _dataset_masses(nums, graphs, directed, loops, table)
    norm = int(sum(masses))
    if table == "dataset_counts":
        assert norm < (1 << 16)
        gt = A.GpuTable(A.Gpu(0), A.Categorical(masses))
        assert gt.paths() & A.ANS_PATH_ENC_LDS and gt.paths() & A.ANS_PATH_DEC_LDS
    ds = A.GpuDenseSets(A.Gpu(0), A.Bernoulli(mass, norm), directed, loops)
    data, offsets, lens = ds.encode(nums, graphs)
    for g, (n, e) in enumerate(zip(nums, graphs)):
        dense = orc.dense_set(e, n, directed, loops)
        od, _, _ = orc.encode_chunks(masses, dense, max(len(dense), 1))
        want = od.tobytes() if len(dense) else bytes(orc.Message.zeros().flatten())
        got = data[int(offsets[g]):int(offsets[g] + lens[g])].tobytes()
        assert got == want, g
        er = A.ErdosRenyi(A.Bernoulli(mass, norm), n, directed, loops)
        m = A.Message.zeros()
        er.push(m, [tuple(map(int, x)) for x in e])
        assert got == m.flatten(), g
    back = ds.decode(nums, data, offsets, lens, cap=5)  # too small: the second pass sizes it
    for g, (n, e) in enumerate(zip(nums, graphs)):
        want = _alphabet_sorted(e, n, directed, loops) if len(e) else np.zeros((0, 2), np.uint32)
        assert np.array_equal(back[g], want), g
    bad = [np.asarray([[3, 1]], np.uint32) if not directed else np.asarray([[70, 1]], np.uint32)] + graphs[1:]
    with pytest.raises(A.AnsError) as e:
        ds.encode(nums, bad)
    assert e.value.code == A.ANS_E_SYMBOL
