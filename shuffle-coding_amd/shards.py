"""Multi-GPU sharding of the bulk path: independent chunks, no collective
on the data path.

Chunks are independent reference messages, so GPU g of G takes the contiguous chunk range
[g*C/G, (g+1)*C/G) of the C chunks, codes it on its own device, and the per-chunk streams
are concatenated in chunk order with global offsets from an exclusive scan of the lengths.
The only communication is the assembly of the container (or of the decoded symbols):

  * the per-rank totals are exchanged (one all_gather of two integers) and scanned, so every
    rank knows where its bytes start in the whole;
  * the bytes then go straight to their final place: into a file every rank maps (`out` =
    a path: each rank writes its own range, no byte crosses the process group), or, in
    memory, by point-to-point sends to rank `dst`, which receives each rank's range into
    one preallocated buffer at its scanned offset, in pieces of at most `piece` bytes.

Nothing is pickled and no rank holds more than its own shard plus (on `dst`) the result, so
an 8 GiB C4 container needs 8 GiB on `dst`, not a gathered copy per rank.  The process group
may be gloo (CPU tensors) or nccl/RCCL (tensors staged through the rank's current device).
"""
import numpy as np

PIECE = 256 << 20  # bytes per point-to-point message


def shard_chunks(nchunks, world, rank):
    """Contiguous, balanced chunk range [c0, c1) of rank `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(nchunks, world)
    c0 = rank * base + min(rank, extra)
    return c0, c0 + base + (1 if rank < extra else 0)


def shard_symbols(n, chunk_len, world, rank):
    """(sym_start, sym_end, chunk_start, chunk_end) of this rank; only the last rank can end
    with the ragged last chunk, so every shard boundary is a chunk boundary."""
    nchunks = -(-n // chunk_len) if n else 0
    c0, c1 = shard_chunks(nchunks, world, rank)
    return min(n, c0 * chunk_len), min(n, c1 * chunk_len), c0, c1


def assemble(shards):
    """shards: list of (data uint8, lens) in rank order -> (data, offsets, lens) of the whole."""
    lens = np.concatenate([np.asarray(l, np.uint64) for _, l in shards]) if shards else np.zeros(0, np.uint64)
    data = np.concatenate([np.asarray(d, np.uint8) for d, _ in shards]) if shards else np.zeros(0, np.uint8)
    return data, exclusive_offsets(lens), lens


def exclusive_offsets(lens):
    offsets = np.zeros(len(lens), np.uint64)
    if len(lens) > 1:
        offsets[1:] = np.cumsum(np.asarray(lens, np.uint64)[:-1], dtype=np.uint64)
    return offsets


def _device(group):
    import torch
    import torch.distributed as dist

    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _all_gather_ints(values, group):
    """Every rank's small int64 vector (same length on all ranks), rank order."""
    import torch
    import torch.distributed as dist

    dev = _device(group)
    t = torch.as_tensor(np.asarray(values, np.int64), device=dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return np.stack([p.cpu().numpy() for p in parts])


def _send_bytes(buf, dst, group, piece):
    import torch
    import torch.distributed as dist

    dev = _device(group)
    flat = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    for a in range(0, len(flat), piece):
        t = torch.from_numpy(flat[a:a + piece]).to(dev)
        dist.send(t, dst=dist.get_global_rank(group, dst) if group is not None else dst, group=group)


def _recv_bytes(out, src, group, piece):
    """Receive len(out) bytes from rank `src` into the uint8 view `out`."""
    import torch
    import torch.distributed as dist

    dev = _device(group)
    peer = dist.get_global_rank(group, src) if group is not None else src
    for a in range(0, len(out), piece):
        m = min(piece, len(out) - a)
        if dev.type == "cpu":
            dist.recv(torch.from_numpy(out[a:a + m]), src=peer, group=group)
        else:
            t = torch.empty(m, dtype=torch.uint8, device=dev)
            dist.recv(t, src=peer, group=group)
            out[a:a + m] = t.cpu().numpy()


def _gather_to(local, counts, starts, out, dst, group, piece):
    """Rank `dst` fills out[starts[r] : starts[r] + counts[r]] with rank r's `local` (a flat
    uint8 view); the other ranks send theirs.  Point-to-point, one rank at a time."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if rank == dst:
        for r in range(world):
            seg = out[starts[r]:starts[r] + counts[r]]
            if r == dst:
                seg[:] = local
            elif counts[r]:
                _recv_bytes(seg, r, group, piece)
    elif len(local):
        _send_bytes(local, dst, group, piece)


def encode_distributed(encode_shard, syms, chunk_len, group=None, dst=0, out=None, piece=PIECE):
    """Each rank encodes its shard of `syms` (the full array, or anything that slices) with
    encode_shard(local_syms, chunk_len) -> (data, offsets, lens), e.g. ans_amd.GpuTable.
    encode_chunks on its own device.

    out=None: rank `dst` returns (data, offsets, lens) of the whole container, the others None.
    out=path (a file every rank can open): the container bytes are written there, each rank
    its own range (rank `dst` sizes the file first); every rank returns (None, offsets, lens)
    of the whole.
    """
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    s0, s1, c0, c1 = shard_symbols(len(syms), chunk_len, world, rank)
    data, _, lens = encode_shard(syms[s0:s1], chunk_len)
    data = np.ascontiguousarray(np.asarray(data, np.uint8)).reshape(-1)
    lens = np.asarray(lens, np.uint64)
    local_total = int(lens.sum()) if len(lens) else 0
    if local_total != len(data):
        raise ValueError("encode_shard returned a container that is not dense")
    sizes = _all_gather_ints([c1 - c0, local_total], group)
    nchunk, nbytes = sizes[:, 0], sizes[:, 1]
    byte_start = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.int64)
    chunk_start = np.concatenate([[0], np.cumsum(nchunk)[:-1]]).astype(np.int64)
    total = int(nbytes.sum())
    # every rank's lengths to every rank (8 bytes per chunk: 16 MB for an 8 GiB C4 container)
    all_lens = np.zeros(int(nchunk.sum()), np.uint64)
    _all_gather_varlen(lens, nchunk, chunk_start, all_lens, group)
    offsets = exclusive_offsets(all_lens)
    if out is not None:
        if rank == dst:
            with open(out, "wb") as f:
                f.truncate(total)
        dist.barrier(group=group)
        if local_total:
            mm = np.memmap(out, dtype=np.uint8, mode="r+", offset=int(byte_start[rank]), shape=(local_total,))
            mm[:] = data
            mm.flush()
            del mm
        dist.barrier(group=group)
        return None, offsets, all_lens
    whole = np.empty(total, np.uint8) if rank == dst else None
    _gather_to(data, nbytes, byte_start, whole, dst, group, piece)
    return (whole, offsets, all_lens) if rank == dst else None


def _all_gather_varlen(local, counts, starts, out, group):
    """out[starts[r] : starts[r] + counts[r]] = rank r's `local` (uint64), on every rank
    (padded all_gather of one flat tensor)."""
    import torch
    import torch.distributed as dist

    dev = _device(group)
    width = int(counts.max()) if len(counts) else 0
    if width == 0:
        return
    pad = np.zeros(width, np.int64)
    pad[:len(local)] = np.asarray(local, np.uint64).view(np.int64)
    t = torch.from_numpy(pad).to(dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    for r, p in enumerate(parts):
        out[starts[r]:starts[r] + counts[r]] = p.cpu().numpy()[:counts[r]].view(np.uint64)


def _dtype_of(kind, itemsize):
    """The numpy dtype of kind character code `kind` (ord of 'u', 'i', 'b' or 'f') and `itemsize`
    bytes: alias types (np.ulonglong, np.intc, ...) gather as their canonical dtype."""
    k = chr(kind)
    if k not in "uibf":
        raise ValueError(f"unexpected decoder dtype kind {k!r}")
    return np.dtype(bool) if k == "b" else np.dtype(f"{k}{itemsize}")


def decode_distributed(decode_shard, data, offsets, lens, n, chunk_len, group=None, dst=0, out=None,
                       dtype=None, piece=PIECE):
    """Inverse of encode_distributed: each rank decodes its chunk range of the container
    (decode_shard(data, offsets, lens, n_local, chunk_len) -> symbols; `data` the whole
    container in memory, or a path to it, which each rank maps and reads its range of).

    out=None: rank `dst` returns the n symbols, the others None.  out=path: the symbols are
    written there (`dtype` elements), each rank its own range; every rank returns None.
    dtype=None: the decoders' own dtype (the widest over the ranks that decoded symbols, agreed
    through one all_gather, as kind and width so alias types agree); a dtype that cannot hold
    every decoded value raises, and so do decoders mixing signed and unsigned 64-bit types.
    (Round 3 changed the default from np.uint8 to None: files written with out=path now hold
    the decoders' element width, e.g. 4 bytes for u32 symbols; pass dtype=np.uint8 for the old one.)
    """
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    s0, s1, c0, c1 = shard_symbols(n, chunk_len, world, rank)
    off = np.asarray(offsets[c0:c1], np.uint64)
    ln = np.asarray(lens[c0:c1], np.uint64)
    base = int(off[0]) if len(off) else 0
    end = int(off[-1] + ln[-1]) if len(off) else 0
    if isinstance(data, (str, bytes)) or hasattr(data, "__fspath__"):
        src = np.memmap(data, dtype=np.uint8, mode="r", offset=base, shape=(end - base,)) if end > base \
            else np.zeros(0, np.uint8)
    else:
        src = np.asarray(data[base:end])
    res = np.asarray(decode_shard(np.asarray(src), off - np.uint64(base), ln, s1 - s0, chunk_len))
    if dtype is None:  # every rank must write the same element width: agree on the decoders' dtype
        info = _all_gather_ints([s1 - s0, ord(res.dtype.kind), res.dtype.itemsize], group)
        found = [_dtype_of(int(k), int(w)) for m, k, w in info if m > 0]
        dtype = np.result_type(*found) if found else res.dtype
        if found and all(f.kind in "uib" for f in found) and dtype.kind == "f":
            # np.result_type(int64, uint64) is float64: no integer type holds both
            raise ValueError(f"decoders disagree on signedness at 64 bits ({sorted(set(map(str, found)))})")
    dtype = np.dtype(dtype)
    local = np.ascontiguousarray(res.astype(dtype, copy=False))
    if res.size and not np.array_equal(local, res):
        raise ValueError(f"decoded symbols do not fit {dtype} (decoder returned {res.dtype})")
    w = dtype.itemsize
    if out is not None:
        if rank == dst:
            with open(out, "wb") as f:
                f.truncate(n * w)
        dist.barrier(group=group)
        if s1 > s0:
            mm = np.memmap(out, dtype=np.uint8, mode="r+", offset=s0 * w, shape=((s1 - s0) * w,))
            mm[:] = local.view(np.uint8).reshape(-1)
            mm.flush()
            del mm
        dist.barrier(group=group)
        return None
    counts = np.array([(shard_symbols(n, chunk_len, world, r)[1] - shard_symbols(n, chunk_len, world, r)[0]) * w
                       for r in range(world)], np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    whole = np.empty(n, dtype) if rank == dst else None
    _gather_to(local.view(np.uint8).reshape(-1), counts, starts,
               None if whole is None else whole.view(np.uint8).reshape(-1), dst, group, piece)
    return whole
