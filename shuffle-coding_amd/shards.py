"""Multi-GPU sharding of the bulk path: independent chunks, no collective
on the data path.

Chunks are independent reference messages, so GPU g of G takes the contiguous chunk range
[g*C/G, (g+1)*C/G) of the C chunks, codes it on its own device, and the per-chunk streams
are concatenated in chunk order with global offsets from an exclusive scan of the lengths.
The only communication is gathering each shard's bytes to the host that assembles the
container; `torch.distributed` is used for that (gloo or nccl/RCCL), never inside a kernel.
"""
import numpy as np


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
    offsets = np.zeros(len(lens), np.uint64)
    if len(lens) > 1:
        offsets[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return data, offsets, lens


def encode_distributed(encode_shard, syms, chunk_len, group=None, dst=0):
    """Each rank encodes its shard of `syms` (the full array, or any object supporting
    slicing) with encode_shard(local_syms, chunk_len) -> (data, offsets, lens), e.g.
    ans_amd.GpuTable.encode_chunks on its own device; rank `dst` returns the assembled
    (data, offsets, lens), other ranks return None."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    s0, s1, _, _ = shard_symbols(len(syms), chunk_len, world, rank)
    data, _, lens = encode_shard(syms[s0:s1], chunk_len)
    gathered = [None] * world if rank == dst else None
    dist.gather_object((np.asarray(data), np.asarray(lens)), gathered, dst=dst, group=group)
    return assemble(gathered) if rank == dst else None


def decode_distributed(decode_shard, data, offsets, lens, n, chunk_len, group=None, dst=0):
    """Inverse of encode_distributed: each rank decodes its chunk range of the container
    (decode_shard(data, offsets, lens, n_local, chunk_len) -> symbols) and rank `dst`
    returns the concatenated symbols."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    s0, s1, c0, c1 = shard_symbols(n, chunk_len, world, rank)
    off = np.asarray(offsets[c0:c1], np.uint64)
    ln = np.asarray(lens[c0:c1], np.uint64)
    base = int(off[0]) if len(off) else 0
    end = int(off[-1] + ln[-1]) if len(off) else 0
    local = decode_shard(np.asarray(data[base:end]), off - np.uint64(base), ln, s1 - s0, chunk_len)
    gathered = [None] * world if rank == dst else None
    dist.gather_object(np.asarray(local), gathered, dst=dst, group=group)
    return np.concatenate(gathered) if rank == dst else None
