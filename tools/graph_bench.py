"""Device-resident throughput of the graph models' bulk caller (ErdosRenyi's DenseSetIID,
C ABI section 5) on one MI355X: edges -> dense indicator vector -> chunked IID<Bernoulli>
encode, and decode -> edges, with the reference's plain_erdos_renyi Bernoulli
(norm 2^28, mass = floor(p * 2^28), src/graph_codec.rs:398-401).

usage: python tools/graph_bench.py [num_nodes=65536] [p=1e-4] [chunk_len=4096] [reps=5]
Prints one JSON line: slot GiB/s (one u8 indicator per alphabet slot) for encode, decode and
the round trip, with the kernel times from HIP events on the context stream's torch wrapper.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    p = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    norm = 1 << 28
    mass = int(p * norm)
    g = A.Gpu(0)
    gt = A.GpuTable(g, A.Bernoulli(mass, norm).categorical)
    space = (n, 0, 0)
    slots = len(A.AllEdgeIndices(n))
    rng = np.random.default_rng(5)
    m = int(rng.binomial(slots, mass / norm))
    i = rng.integers(0, n, 3 * m // 2 + 16)
    j = rng.integers(0, n, 3 * m // 2 + 16)
    a, b = np.minimum(i, j), np.maximum(i, j)
    e = np.unique(np.stack([a, b], 1)[a != b], axis=0)[:m].astype(np.uint32)
    e = e[np.lexsort((e[:, 0], e[:, 1]))]  # alphabet order: by j, then i (src/graph_codec.rs:192)
    m = len(e)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    d_edges = torch.from_numpy(e.view(np.int32)).cuda()
    d_dense = torch.empty(slots + 16, dtype=torch.uint8, device="cuda")
    d_back = torch.empty(slots + 16, dtype=torch.uint8, device="cuda")
    nch = -(-slots // L)
    cap = gt.slot_capacity(L)
    d_slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
    d_lens = torch.empty(nch, dtype=torch.int32, device="cuda")
    d_status = torch.zeros(4, dtype=torch.int32, device="cuda")
    d_out = torch.empty(m + 16, 2, dtype=torch.int32, device="cuda")
    d_count = torch.zeros(2, dtype=torch.int64, device="cuda")
    lib = A.lib()

    def enc():
        A._check(lib.ans_dev_edges_to_dense(g.h, *space, d_edges.data_ptr(), m, d_dense.data_ptr(),
                                            d_status.data_ptr(), sp), "edges_to_dense")
        gt.dev_encode(d_dense, 1, slots, L, d_slots, cap, d_lens, d_status, stream)

    def dec():
        gt.dev_decode(d_slots, None, cap, d_lens, slots, L, d_back, 1, d_status, stream)
        A._check(lib.ans_dev_dense_to_edges(g.h, *space, d_back.data_ptr(), d_out.data_ptr(), m + 16,
                                            d_count.data_ptr(), d_status.data_ptr(), sp), "dense_to_edges")

    te, td = [], []
    for r in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record(stream)
        enc()
        ev[1].record(stream)
        dec()
        ev[2].record(stream)
        torch.cuda.synchronize()
        if r:
            te.append(ev[0].elapsed_time(ev[1]) / 1e3)
            td.append(ev[1].elapsed_time(ev[2]) / 1e3)
    assert g.status(d_status, stream) == 0
    assert int(d_count[0].item()) == m
    got = d_out[:m].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, e), "edges differ after the round trip"
    comp = int(d_lens.to(torch.int64).sum().item())
    t_e, t_d = float(np.median(te)), float(np.median(td))
    print(json.dumps({
        "workload": f"ErdosRenyi dense set, undirected n={n} ({slots} slots), p={p} (mass {mass}/2^28), "
                    f"{m} edges, chunk_len {L}",
        "encode_ms": round(1e3 * t_e, 4), "decode_ms": round(1e3 * t_d, 4),
        "slot_gib_s_encode": slots / t_e / 2**30, "slot_gib_s_decode": slots / t_d / 2**30,
        "slot_gib_s_round_trip": slots / (t_e + t_d) / 2**30,
        "compressed_bytes": comp, "bits_per_edge": 8 * comp / max(m, 1),
        "ideal_bits_per_edge": float(slots * (-(p * np.log2(p)) - (1 - p) * np.log2(1 - p)) / max(m, 1)),
    }))


if __name__ == "__main__":
    main()
