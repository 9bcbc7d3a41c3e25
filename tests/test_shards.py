"""The N>1 path: chunk sharding across ranks on CPU with gloo, world_size 2.

Each rank codes its contiguous chunk range; the container is assembled either in rank 0's
memory (point-to-point pieces at scanned offsets) or in one file each rank writes its own
range of.  The result must equal one process coding everything (chunk streams are
independent messages).  The
per-shard coder here is the oracle standing in for GpuTable.encode_chunks/decode_chunks
(no GPU in this container); the GPU versions of those calls are covered by
tests/test_gpu_parity.py.
"""
import os
import socket

import numpy as np
import pytest

import shards
from oracle import oracle as orc


def test_shard_ranges_cover_every_chunk_once():
    for nchunks in (0, 1, 7, 64, 1000):
        for world in (1, 2, 3, 8):
            got = [shards.shard_chunks(nchunks, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == nchunks
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    # symbol ranges end on chunk boundaries; only the last rank holds the ragged chunk
    n, L = 10_007, 100
    ranges = [shards.shard_symbols(n, L, 3, r) for r in range(3)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(r[1] % L == 0 for r in ranges[:-1])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, masses, syms, chunk_len, q, mode, tmp):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        enc = lambda s, L: orc.encode_chunks(masses, s, L)  # noqa: E731
        dec = lambda d, o, l, n, L: orc.decode_chunks(masses, d, o, l, n, L)  # noqa: E731
        if mode == "file":  # every rank writes its own range of one container file
            path = os.path.join(tmp, "container.bin")
            _, offsets, lens = shards.encode_distributed(enc, syms, chunk_len, out=path)
            sym_path = os.path.join(tmp, "symbols.bin")
            shards.decode_distributed(dec, path, offsets, lens, len(syms), chunk_len, out=sym_path)
            if rank == 0:
                with open(path, "rb") as f:
                    data = f.read()
                q.put(("enc", data, offsets.tolist(), lens.tolist()))
                # dtype=None: the file holds the decoder's own elements (the oracle's uint32)
                q.put(("dec", np.fromfile(sym_path, np.uint32).tolist()))
            return
        # in memory: point-to-point pieces of 1000 bytes into rank 0's preallocated buffers
        got = shards.encode_distributed(enc, syms, chunk_len, piece=1000)
        if rank == 0:
            data, offsets, lens = got
            q.put(("enc", data.tobytes(), offsets.tolist(), lens.tolist()))
        else:
            data = offsets = lens = None
        obj = [data, offsets, lens]
        dist.broadcast_object_list(obj, src=0)
        back = shards.decode_distributed(dec, obj[0], obj[1], obj[2], len(syms), chunk_len, piece=1000)
        if rank == 0:
            q.put(("dec", back.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["memory", "file"])
@pytest.mark.parametrize("n,chunk_len,nsym", [(50_000, 4096, 256), (4096 * 5, 4096, 256), (999, 10, 256), (5, 10, 256),
                                              (30_000, 4096, 65_536)])
def test_two_rank_gloo_matches_single_process(n, chunk_len, nsym, mode, tmp_path):
    # nsym 65,536: symbols above 255 survive the assembly (no cast to an 8-bit default dtype)
    import torch.multiprocessing as mp

    masses = np.asarray([1 + (i * 7919) % 4000 for i in range(nsym)], np.uint64)
    syms = orc.gen_iid(masses, 11, 0, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, masses, syms, chunk_len, q, mode, str(tmp_path)))
             for r in range(2)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    results = {m[0]: m[1:] for m in msgs}
    ref_data, ref_off, ref_lens = orc.encode_chunks(masses, syms, chunk_len)
    data, offsets, lens = results["enc"]
    assert data == ref_data.tobytes()
    assert offsets == ref_off.tolist() and lens == ref_lens.tolist()
    assert results["dec"][0] == syms.tolist()
    if nsym > 256:
        assert max(results["dec"][0]) > 255


def test_decode_dtype_that_loses_values_raises():
    dec = lambda d, o, l, n, L: np.array([3, 300], np.uint32)  # noqa: E731

    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already up")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with pytest.raises(ValueError, match="do not fit"):
            shards.decode_distributed(dec, np.zeros(4, np.uint8), np.zeros(1, np.uint64), np.full(1, 4, np.uint64),
                                      2, 10, dtype=np.uint8)
        got = shards.decode_distributed(dec, np.zeros(4, np.uint8), np.zeros(1, np.uint64), np.full(1, 4, np.uint64),
                                        2, 10)
        assert got.dtype == np.uint32 and got.tolist() == [3, 300]
    finally:
        dist.destroy_process_group()


def _gpu_worker(rank, world, port, masses, syms, chunk_len, q):
    import torch.distributed as dist

    import ans_amd as A

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        table = A.GpuTable(A.Gpu(0), A.Categorical(masses))  # both ranks share the one GPU here
        got = shards.encode_distributed(table.encode_chunks, syms, chunk_len)
        obj = list(got) if rank == 0 else [None, None, None]
        dist.broadcast_object_list(obj, src=0)
        dec = lambda d, o, l, n, L: table.decode_chunks(d, o, l, n, L, np.uint8)  # noqa: E731
        back = shards.decode_distributed(dec, obj[0], obj[1], obj[2], len(syms), chunk_len)
        if rank == 0:
            q.put((obj[0].tobytes(), obj[2].tolist(), back.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_sharded_gpu_coding_matches_oracle():
    import torch.multiprocessing as mp

    import ans_amd as A

    masses = A.c3_masses()
    n, chunk_len = 1000 * 4096 + 77, 4096
    syms = orc.gen_iid(masses, 5, 0, n).astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, masses, syms, chunk_len, q)) for r in range(2)]
    for p in procs:
        p.start()
    data, lens, back = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref_data, _, ref_lens = orc.encode_chunks(masses, syms, chunk_len)
    assert data == ref_data.tobytes() and lens == ref_lens.tolist()
    assert back == syms.tolist()
