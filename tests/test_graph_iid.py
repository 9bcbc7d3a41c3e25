"""GraphIID<NodeC, EdgeC, ErdosRenyi> with labels (src/graph_codec.rs:19-94): the model the
reference's --er / --uniform-er runs on node- and edge-labelled datasets (Independent of one
GraphIID per graph, src/benchmark.rs:308-372, count-built label Categoricals and the dataset
Bernoulli, src/benchmark.rs:549-578).

CPU: the host mirror (ans_amd.GraphIID on one Message) against the oracle's literal composition
(oracle.graph_iid_push / graph_iid_pop: EdgesIID::push = sorted labels then the indicator vector,
then the node labels), and the Uniform-as-all-ones-Categorical substitution the GPU table set uses.
GPU (`gpu` marker): ans_gpu_graphs_encode / _decode through the C ABI on a MUTAG-shaped synthetic
dataset (188 graphs, 10-28 nodes, 7 node labels, 4 edge labels; the TU dataset itself is a download
the reference makes, src/datasets.rs, not available here), every graph's stream byte-equal to the
oracle's message of that graph; and Independent over variable-length chunks against the oracle.
"""
import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

NODE_P = [0.72, 0.10, 0.12, 0.02, 0.02, 0.01, 0.01]  # MUTAG-like label frequencies (7 node labels)
EDGE_P = [0.52, 0.04, 0.40, 0.04]  # 4 bond types


def _molecule(rng, n, directed, loops):
    """A sparse connected-ish graph: a random tree plus a few extra pairs, in the alphabet."""
    pairs = set()
    for v in range(1, n):
        u = int(rng.integers(0, v))
        pairs.add((u, v))
    for _ in range(n // 6):
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b:
            pairs.add((min(a, b), max(a, b)))
    if loops and n:
        for v in rng.choice(n, size=min(n, 2), replace=False):
            pairs.add((int(v), int(v)))
    edges = []
    for i, j in sorted(pairs):
        if directed and i != j and rng.random() < 0.5:
            i, j = j, i
        edges.append((i, j))
    rng.shuffle(edges)  # any order in, sorted by index out
    return np.asarray(edges, dtype=np.uint32).reshape(-1, 2)


def _dataset(seed, num_graphs=188, directed=False, loops=False, lo=10, hi=29, extra=()):
    rng = np.random.default_rng(seed)
    nums = [int(x) for x in rng.integers(lo, hi, num_graphs)] + list(extra)
    graphs = []
    for n in nums:
        e = _molecule(rng, n, directed, loops)
        nl = rng.choice(len(NODE_P), size=n, p=NODE_P).astype(np.uint32)
        el = rng.choice(len(EDGE_P), size=len(e), p=EDGE_P).astype(np.uint32)
        graphs.append((n, nl, e, el))
    return graphs


def _counts(values):
    """DatasetStats::dist (src/benchmark.rs:576-579): masses 0..=max label, the counts."""
    v = np.concatenate([np.asarray(x, dtype=np.int64) for x in values])
    return np.bincount(v, minlength=int(v.max()) + 1).astype(np.uint64)


def _stats(graphs, directed, loops):
    """DatasetStats::edge_labelled (src/benchmark.rs:549-566): Bernoulli(total_edges,
    total_possible_edges) and the node / edge label Categoricals."""
    total_edges = sum(len(g[2]) for g in graphs)
    possible = sum(len(orc.all_edge_indices(g[0], directed, loops)) for g in graphs)
    bern = [possible - total_edges, total_edges]
    return bern, _counts([g[1] for g in graphs]), _counts([g[3] for g in graphs])


def _oracle_stream(g, bern, node, edge, directed, loops):
    n, nl, e, el = g
    m = orc.Message.zeros()
    assert orc.graph_iid_push(m, n, nl, e, el, bern, node, edge, directed, loops) == 0
    return m.flatten()


def _host_graph(g, with_nodes=True, with_edges=True):
    n, nl, e, el = g
    return A.Graph([int(x) for x in nl] if with_nodes else [None] * n,
                   [((int(a), int(b)), int(l) if with_edges else None) for (a, b), l in zip(e, el)])


def _sorted_edges(e, el):
    order = sorted(range(len(e)), key=lambda k: (int(e[k][0]), int(e[k][1])))
    return np.asarray([e[k] for k in order], dtype=np.uint32).reshape(-1, 2), np.asarray([el[k] for k in order],
                                                                                        dtype=np.uint32)


# ---------------------------------------------------------------- host mirror (CPU)
@pytest.mark.parametrize("directed,loops", [(False, False), (True, False), (False, True), (True, True)])
def test_host_graph_iid_matches_oracle_composition(directed, loops):
    graphs = _dataset(5 + 2 * directed + loops, num_graphs=6, directed=directed, loops=loops, lo=0, hi=14,
                      extra=(0, 1, 2))
    bern, nodes, edges = _stats(graphs, directed, loops)
    for g in graphs:
        n = g[0]
        codec = A.GraphIID(n, A.ErdosRenyi(A.Bernoulli(int(bern[1]), int(sum(bern))), n, directed, loops),
                           A.Categorical(nodes), A.Categorical(edges))
        m = A.Message.zeros()
        codec.push(m, _host_graph(g))
        want = _oracle_stream(g, bern, ("cat", nodes), ("cat", edges), directed, loops)
        assert m.flatten() == want
        back = codec.pop(m)
        se, sl = _sorted_edges(g[2], g[3])
        assert back.node_labels == [int(x) for x in g[1]]
        assert back.edges == [((int(a), int(b)), int(l)) for (a, b), l in zip(se, sl)]
        assert m == A.Message.zeros()
        # the oracle's pop of the same bytes
        om = orc.Message.unflatten(want)
        on, oe, ol = orc.graph_iid_pop(om, n, bern, ("cat", nodes), ("cat", edges), directed, loops)
        assert on == [int(x) for x in g[1]] and oe == [tuple(map(int, x)) for x in se] and ol == [int(x) for x in sl]
        codec.test(back, A.Message.zeros())  # Codec::test (src/ans.rs:47-68)


def test_host_graph_iid_empty_codecs_and_uniform_labels():
    """EmptyCodec nodes / edges code nothing (the unlabelled GraphIID = ErdosRenyi alone);
    Uniform labels (--uniform-er) equal the all-ones Categorical the GPU set holds."""
    graphs = _dataset(9, num_graphs=4, lo=3, hi=12)
    bern, nodes, edges = _stats(graphs, False, False)
    b = A.Bernoulli(int(bern[1]), int(sum(bern)))
    for g in graphs:
        n = g[0]
        plain = A.GraphIID(n, A.ErdosRenyi(b, n))
        m = A.Message.zeros()
        plain.push(m, _host_graph(g, with_nodes=False, with_edges=False))
        assert m.flatten() == _oracle_stream(g, bern, None, None, False, False)
        un, ue = A.Uniform(len(nodes)), A.Uniform(len(edges))
        uni = A.GraphIID(n, A.ErdosRenyi(b, n), un, ue)
        m = A.Message.zeros()
        uni.push(m, _host_graph(g))
        want = _oracle_stream(g, bern, ("uniform", len(nodes)), ("uniform", len(edges)), False, False)
        assert m.flatten() == want
        ones = _oracle_stream(g, bern, ("cat", np.ones(len(nodes), np.uint64)), ("cat", np.ones(len(edges), np.uint64)),
                              False, False)
        assert ones == want
        back = uni.pop(m)
        assert back.node_labels == [int(x) for x in g[1]]


def test_host_graph_iid_rejects_edges_outside_the_alphabet():
    codec = A.GraphIID(4, A.ErdosRenyi(A.Bernoulli(3, 10), 4), A.Categorical([1, 1]), A.Categorical([1, 1]))
    with pytest.raises(A.AnsError):
        codec.push(A.Message.zeros(), A.Graph([0, 1, 0, 1], [((2, 1), 0)]))  # undirected: (1, 2) only


# ---------------------------------------------------------------- GPU
def _check_dataset(graphs, bern, node, edge, directed, loops, node_codec, edge_codec, cap=None):
    gg = A.GpuGraphs(A.Gpu(0), A.Bernoulli(int(bern[1]), int(sum(bern))), node_codec, edge_codec, directed, loops)
    enc = [(g[0], g[1] if node is not None else None, g[2], g[3] if edge is not None else None) for g in graphs]
    data, offsets, lens = gg.encode(enc)
    assert len(lens) == len(graphs)
    for k, g in enumerate(graphs):
        got = data[int(offsets[k]):int(offsets[k] + lens[k])].tobytes()
        assert got == _oracle_stream(g, bern, node, edge, directed, loops), k
    back = gg.decode([g[0] for g in graphs], data, offsets, lens, cap=cap)
    for k, (g, (bn, be, bl)) in enumerate(zip(graphs, back)):
        se, sl = _sorted_edges(g[2], g[3])
        assert np.array_equal(be, se), k
        if node is not None:
            assert np.array_equal(bn, g[1]), k
        if edge is not None:
            assert np.array_equal(bl, sl), k
    return gg, data, offsets, lens


@pytest.mark.gpu
def test_gpu_graphs_mutag_shaped_bit_exact():
    """The reference's default --er model on an edge-labelled dataset (src/benchmark.rs:308-316):
    count-built node / edge Categoricals and Bernoulli(total_edges, total_possible_edges), all
    norms below 2^16, a set the fast Independent kernels take."""
    graphs = _dataset(188)
    bern, nodes, edges = _stats(graphs, False, False)
    assert sum(bern) < (1 << 16) and nodes.sum() < (1 << 16) and edges.sum() < (1 << 16)
    gg, data, _, _ = _check_dataset(graphs, bern, ("cat", nodes), ("cat", edges), False, False,
                                    A.Categorical(nodes), A.Categorical(edges))
    assert gg.fast() in (1, 2)
    # the host mirror codes the same bytes (one graph)
    g = graphs[7]
    codec = A.GraphIID(g[0], A.ErdosRenyi(A.Bernoulli(int(bern[1]), int(sum(bern))), g[0]), A.Categorical(nodes),
                       A.Categorical(edges))
    m = A.Message.zeros()
    codec.push(m, _host_graph(g))
    assert m.flatten() == _oracle_stream(g, bern, ("cat", nodes), ("cat", edges), False, False)


@pytest.mark.gpu
@pytest.mark.parametrize("directed,loops", [(True, False), (False, True), (True, True)])
def test_gpu_graphs_directed_loops(directed, loops):
    graphs = _dataset(21 + 2 * directed + loops, num_graphs=60, directed=directed, loops=loops, lo=0, hi=24,
                      extra=(0, 1, 2, 40))
    bern, nodes, edges = _stats(graphs, directed, loops)
    _check_dataset(graphs, bern, ("cat", nodes), ("cat", edges), directed, loops, A.Categorical(nodes),
                   A.Categorical(edges), cap=7)  # too small: the second pass sizes it


@pytest.mark.gpu
def test_gpu_graphs_node_labelled_and_uniform():
    """--er on a node-labelled dataset (src/benchmark.rs:349-358: EmptyCodec edges) and
    --uniform-er (Uniform(size) labels, src/benchmark.rs:318-330)."""
    graphs = _dataset(33, num_graphs=50)
    bern, nodes, edges = _stats(graphs, False, False)
    _check_dataset(graphs, bern, ("cat", nodes), None, False, False, A.Categorical(nodes), None)
    _check_dataset(graphs, bern, ("uniform", len(nodes)), ("uniform", len(edges)), False, False,
                   A.Uniform(len(nodes)), A.Uniform(len(edges)))
    _check_dataset(graphs, bern, None, None, False, False, None, None)  # plain ErdosRenyi


@pytest.mark.gpu
def test_gpu_graphs_wide_and_large_norm_tables():
    """Label tables outside the fast set's range: a 300-symbol node table and a 2^30-norm ER
    Bernoulli (plain_erdos_renyi's 2^28 style), still bit-exact (the exact lane coder)."""
    rng = np.random.default_rng(44)
    graphs = _dataset(45, num_graphs=40)
    graphs = [(n, rng.integers(0, 300, n).astype(np.uint32), e, el) for n, _, e, el in graphs]
    bern = [(1 << 30) - (1 << 27), 1 << 27]
    nodes = (1 + rng.integers(0, 1000, 300)).astype(np.uint64)
    _, _, edges = _stats(graphs, False, False)
    _check_dataset(graphs, bern, ("cat", nodes), ("cat", edges), False, False, A.Categorical(nodes),
                   A.Categorical(edges))


@pytest.mark.gpu
def test_gpu_graphs_errors():
    graphs = _dataset(3, num_graphs=5)
    bern, nodes, edges = _stats(graphs, False, False)
    gg = A.GpuGraphs(A.Gpu(0), A.Bernoulli(int(bern[1]), int(sum(bern))), A.Categorical(nodes), A.Categorical(edges))
    n, nl, e, el = graphs[0]
    for bad in ([(n, nl, np.asarray([[2, 1]]), np.asarray([0]))],  # (2, 1): undirected pairs have i < j
                [(n, nl, np.asarray([[0, 1], [0, 1]]), np.asarray([0, 1]))],  # one pair twice
                [(n, nl, np.asarray([[0, 1]]), np.asarray([len(edges)]))],  # label outside the table
                [(n, np.full(n, len(nodes), np.uint32), e, el)]):
        with pytest.raises(A.AnsError) as err:
            gg.encode(bad)
        assert err.value.code == A.ANS_E_SYMBOL
    data, offsets, lens = gg.encode(graphs)
    # a truncated stream under Message::empty() is exhaustion, not a silent decode
    with pytest.raises(A.AnsError) as err:
        gg.decode([g[0] for g in graphs], data, offsets, np.maximum(lens, 1) - 1, gen_kind=A.GEN_EMPTY)
    assert err.value.code in (A.ANS_E_EXHAUSTED, A.ANS_E_MISMATCH)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [A.GEN_ZEROS, A.GEN_RANDOM])
def test_gpu_independent_var_chunks(kind):
    """Independent<Categorical> over variable-length chunks vs the oracle, chunk by chunk."""
    rng = np.random.default_rng(12 + kind)
    tables = [(1 + rng.integers(0, 500, k)).astype(np.uint64) for k in (2, 7, 40, 256)]
    ts = A.GpuTableSet(A.Gpu(0), [A.Categorical(t) for t in tables])
    lens_ = [int(x) for x in rng.integers(0, 3000, 70)] + [0, 1, 5000]
    starts = np.concatenate([[0], np.cumsum(lens_)]).astype(np.uint64)
    n = int(starts[-1])
    tids = rng.integers(0, len(tables), n).astype(np.uint32)
    syms = np.asarray([rng.integers(0, len(tables[t])) for t in tids], dtype=np.uint32)
    data, offsets, lens = ts.encode_var_chunks(tids, syms, starts, gen_kind=kind, seed=9)
    for c in range(len(lens_)):
        a, b = int(starts[c]), int(starts[c + 1])
        if b == a:
            want = (orc.Message.zeros() if kind == A.GEN_ZEROS else orc.Message.random(9 + c)).flatten()
        else:
            want, _, _ = orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, syms[a:b], b - a, tables=tables,
                                                 tids=tids[a:b], kind=kind, seed=9 + c)
            want = want.tobytes()
        assert data[int(offsets[c]):int(offsets[c] + lens[c])].tobytes() == want, c
    back = ts.decode_var_chunks(tids, data, offsets, lens, starts, gen_kind=kind, seed=9)
    assert np.array_equal(back, syms)
