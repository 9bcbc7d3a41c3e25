"""GPU parity: the HIP path (through the C ABI) against the oracle and golden vectors.

Bit-exact is the bar: every chunk's stream must equal the reference message's flattened
bytes (src/ans.rs:255-260) for the same input and chunk boundaries, and decode must be
lossless and return each message to Message::zeros() (src/ans.rs:55-57).
"""
import hashlib

import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    return A.Gpu(0)


def _roundtrip_vs_oracle(gpu, masses, syms, chunk_len, dtype):
    cat = A.Categorical(masses)
    gt = A.GpuTable(gpu, cat)
    s = np.asarray(syms).astype(dtype)
    data, offsets, lens = gt.encode_chunks(s, chunk_len)
    odata, ooffsets, olens = orc.encode_chunks(masses, np.asarray(syms, np.uint32), chunk_len)
    assert np.array_equal(lens, olens)
    assert np.array_equal(offsets, ooffsets)
    assert data.tobytes() == odata.tobytes()
    back = gt.decode_chunks(data, offsets, lens, len(s), chunk_len, dtype)
    assert np.array_equal(back, s)
    return data, lens


# ---------------------------------------------------------------- C1 / C2 (multiset fixtures)
@pytest.mark.parametrize("size", [1000, 10000, 100000])
@pytest.mark.parametrize("layout", ["single_chunk", "chunks64"])
def test_multiset_fixtures_bit_exact(gpu, size, layout, multiset_masses, multiset_vectors, golden_multiset):
    rec = golden_multiset["vectors"][str(size)][layout]
    syms = multiset_vectors[size]
    for dtype in (np.uint16, np.uint32):
        data, lens = _roundtrip_vs_oracle(gpu, multiset_masses, syms, rec["chunk_len"], dtype)
        assert [int(x) for x in lens] == rec["lens"]
        assert hashlib.sha256(data.tobytes()).hexdigest() == rec["sha256"]
        if "hex" in rec:
            assert data.tobytes().hex() == rec["hex"]


def test_golden_small_cases(gpu, golden_small):
    for case in golden_small:
        for dtype in (np.uint8, np.uint16, np.uint32):
            if dtype == np.uint8 and len(case["masses"]) > 256:
                continue
            data, lens = _roundtrip_vs_oracle(gpu, case["masses"], case["syms"], case["chunk_len"], dtype)
            assert data.tobytes().hex() == case["hex"], case["name"]


# ---------------------------------------------------------------- randomized tables
def _random_case(rng, nsym, lo, hi, zero_frac, n):
    masses = rng.integers(lo, hi, size=nsym, dtype=np.int64).astype(np.uint64)
    if zero_frac:
        masses[rng.random(nsym) < zero_frac] = 0
        masses[rng.integers(0, nsym)] = max(1, int(masses.max()))
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    syms = rng.choice(nz, size=n, p=p / p.sum()).astype(np.uint32)
    return masses, syms


@pytest.mark.parametrize("nsym,lo,hi,zero_frac,chunk_len,n", [
    (2, 1, 10, 0.0, 7, 1000),                   # Bernoulli-sized, tiny norm: generic path
    (8, 0, 4, 0.3, 5, 777),                     # zero masses, norm < 2^16
    (256, 1, 1 << 20, 0.0, 4096, 300_000),      # C3-like, fast path, LDS table
    (256, 1, 1 << 20, 0.1, 1563, 100_000),      # zero masses inside the fast path
    (1024, 1 << 10, 1 << 21, 0.0, 1, 3000),     # one symbol per chunk
    (4096, 1, 1 << 12, 0.0, 999, 200_000),      # LDS-sized large alphabet
    (65536, 1, 1 << 12, 0.0, 4096, 400_000),    # C4 alphabet: table from global memory
    (300, 1 << 22, 1 << 24, 0.0, 512, 50_000),  # norm > 2^31: the wide kNormBig kernels
    (3, 1, 2, 0.0, 100, 1000),                  # norm 3..6
    # fast-kernel shapes (chunk_len * width a multiple of 16, >= 512 chunks, ragged tail)
    (256, 1, 1 << 20, 0.0, 64, 100_003),
    (256, 1, 1 << 20, 0.2, 256, 300_017),       # zero masses inside the fast path
    (200, 1 << 8, 1 << 22, 0.0, 1024, 600_000),  # nsym < 256: clamp sentinel
    (17, 1 << 14, 1 << 15, 0.0, 512, 400_000),  # very skewed bytes/symbol (kmax 2)
    (256, 1, 1 << 8, 0.0, 128, 200_000),        # norm ~2^15: generic path for every chunk
    (256, 1, 1 << 23, 0.0, 2048, 1_000_000),    # norm ~2^31: top of the fast range
])
def test_random_tables_bit_exact(gpu, nsym, lo, hi, zero_frac, chunk_len, n):
    rng = np.random.default_rng(nsym * 7919 + n)
    masses, syms = _random_case(rng, nsym, lo, hi, zero_frac, n)
    dtypes = [np.uint32, np.uint16] + ([np.uint8] if nsym <= 256 else [])
    for dtype in dtypes:
        _roundtrip_vs_oracle(gpu, masses, syms, chunk_len, dtype)


@pytest.mark.parametrize("which", ["c3", "c3p2", "wide_masses", "zeros", "top_of_range", "tiny_masses", "shift_18",
                                   "shift_19"])
def test_u_domain_decoder_bit_exact(gpu, which):
    """The fix-up-free decoder (ans_fast.hpp kModeU: u = head - q_m * norm in [0, 2 norm) over a
    512-symbol virtual alphabet) on 256-symbol tables across the fast range: every chunk's bytes
    equal the oracle's and decoding is lossless; the tables expected to build u-domain buckets
    report ANS_PATH_DEC_U (a table whose buckets would need a fourth candidate keeps the r02
    rows, also bit-exact)."""
    rng = np.random.default_rng(sum(map(ord, which)))
    if which == "c3":
        masses = A.c3_masses()
    elif which == "c3p2":
        masses = A.c3_pow2_masses()
    elif which == "wide_masses":
        masses = rng.integers(1, 1 << 20, 256).astype(np.uint64)
    elif which == "zeros":
        masses = rng.integers(1, 1 << 18, 256).astype(np.uint64)
        masses[rng.choice(256, 60, replace=False)] = 0
    elif which == "top_of_range":  # norm just below 2^31
        masses = rng.integers(1 << 21, 1 << 23, 256).astype(np.uint64)
        masses = (masses * ((1 << 31) - 1) // int(masses.sum())).astype(np.uint64)
        masses[masses == 0] = 1
    elif which in ("shift_18", "shift_19"):  # bucket width 2^18 (the widest whose threshold words,
        # below 2^31 since r06, leave the 13 row-address bits to s0) and 2^19 (norm above ~4e8:
        # the r02 rows instead)
        target = 400_000_000 if which == "shift_18" else 800_000_000
        masses = rng.integers(1 << 20, 1 << 23, 256).astype(np.uint64)
        masses = (masses * target // int(masses.sum())).astype(np.uint64)
    else:  # masses of a few units beside large ones: kmax 4, half-unit points
        masses = np.concatenate([rng.integers(1, 4, 16), rng.integers(1 << 12, 1 << 16, 240)]).astype(np.uint64)
    assert int(masses.sum()) < (1 << 31)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    if which in ("c3", "c3p2", "shift_18"):  # (random tables may hold crowded buckets: kModeFar / kModeRows)
        assert gt.paths() & A.ANS_PATH_DEC_U, hex(gt.paths())
    if which == "shift_19":
        assert not gt.paths() & A.ANS_PATH_DEC_U, hex(gt.paths())
    n = 300 * 4096 + 777
    syms = orc.gen_iid(masses, 5, 0, n)
    _roundtrip_vs_oracle(gpu, masses, syms, 4096, np.uint8)


@pytest.mark.parametrize("seed", [0, 1])
def test_fast_decoder_crowded_buckets(gpu, seed):
    """Hundreds of cdf boundaries inside one decode bucket (the bucket table resolves four;
    the rest scan the staged cdf table), symbols drawn uniformly so those are hit often."""
    rng = np.random.default_rng(seed)
    masses = np.ones(256, np.uint64)
    masses[rng.choice(256, 6, replace=False)] = 1 << 22
    masses[rng.choice(256, 40, replace=False)] += rng.integers(0, 2000, 40).astype(np.uint64)
    syms = rng.integers(0, 256, size=520 * 4096 + 99).astype(np.uint32)
    for dtype in (np.uint8, np.uint16, np.uint32):
        _roundtrip_vs_oracle(gpu, masses, syms, 4096, dtype)


def test_ragged_and_empty_inputs(gpu):
    masses = [5, 9, 1, 300000, 17]
    rng = np.random.default_rng(5)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    for n, chunk_len in [(0, 4), (1, 4), (3, 4), (4, 4), (5, 4), (4097, 4096), (10, 1000)]:
        syms = rng.integers(0, 5, size=n).astype(np.uint32)
        data, offsets, lens = gt.encode_chunks(syms, chunk_len)
        od, oo, ol = orc.encode_chunks(masses, syms, chunk_len)
        assert data.tobytes() == od.tobytes() and np.array_equal(lens, ol)
        assert np.array_equal(gt.decode_chunks(data, offsets, lens, n, chunk_len), syms)


def test_device_errors_mirror_reference_panics(gpu):
    gt = A.GpuTable(gpu, A.Categorical([3, 0, 2]))
    with pytest.raises(A.AnsError) as e:
        gt.encode_chunks(np.array([0, 1, 2], np.uint32), 2)  # src/ans.rs:98
    assert e.value.code == A.ANS_E_ZERO_MASS
    with pytest.raises(A.AnsError) as e:
        gt.encode_chunks(np.array([0, 3, 2], np.uint32), 2)  # src/codec.rs:63
    assert e.value.code == A.ANS_E_SYMBOL
    syms = np.array([0, 2, 2, 0, 2, 0, 0, 2], np.uint32)
    data, offsets, lens = gt.encode_chunks(syms, 8)
    # a truncated stream under Message::empty() exhausts the tail (src/ans.rs:144)
    with pytest.raises(A.AnsError) as e:
        gt.decode_chunks(data[1:], offsets, lens - 1, 8, 8, gen_kind=A.GEN_EMPTY)
    assert e.value.code == A.ANS_E_EXHAUSTED
    # ... and under Message::zeros() it does not return to the initial message (src/ans.rs:56)
    with pytest.raises(A.AnsError) as e:
        gt.decode_chunks(data[1:], offsets, lens - 1, 8, 8)
    assert e.value.code == A.ANS_E_MISMATCH
    # norm >= 2^32 codes on the exact 64-bit kernels; only the u32 sampler refuses it
    wide = A.GpuTable(gpu, A.Categorical([1 << 31, 1 << 31]))
    data, offsets, lens = wide.encode_chunks(syms % 2, 4)
    assert np.array_equal(wide.decode_chunks(data, offsets, lens, 8, 4), syms % 2)
    with pytest.raises(A.AnsError) as e:
        wide.sample_chunks(1, 8, 4)
    assert e.value.code == A.ANS_E_NORM_RANGE
    with pytest.raises(A.AnsError) as e:
        A.GpuTable(gpu, A.Categorical([1 << 56, 1]))  # norm > 2^56 breaks the head interval
    assert e.value.code == A.ANS_E_NORM_RANGE


@pytest.mark.parametrize("which", ["generic", "fast"])
def test_corrupt_containers_end_with_an_error(gpu, which):
    """Streams that are empty or all zero bytes under Message::zeros() never reach the head
    interval: decode must end with ANS_E_MISMATCH (the reference's assert_eq!(initial, m),
    src/ans.rs:56), not pull zeros forever; under Message::empty() it is ANS_E_EXHAUSTED
    (src/ans.rs:144).  A slot-layout length past its slot is refused with ANS_E_LEN."""
    torch = pytest.importorskip("torch")
    if which == "generic":  # norm < 2^16 and a ragged chunk: the generic kernels
        masses, n, chunk_len, sym_bytes = [5, 9, 1, 300, 17], 10, 4, 1
    else:  # C3 table, full chunks: the fast kernels
        masses, n, chunk_len, sym_bytes = A.c3_masses(), 4 * 4096, 4096, 1
    gt = A.GpuTable(gpu, A.Categorical(masses))
    nchunks = -(-n // chunk_len)
    for nbytes in (0, 8, 40):
        data = np.zeros(max(1, nchunks * nbytes), np.uint8)
        offsets = np.arange(nchunks, dtype=np.uint64) * nbytes
        lens = np.full(nchunks, nbytes, np.uint64)
        with pytest.raises(A.AnsError) as e:
            gt.decode_chunks(data, offsets, lens, n, chunk_len, np.uint8)
        assert e.value.code == A.ANS_E_MISMATCH, nbytes
        with pytest.raises(A.AnsError) as e:
            gt.decode_chunks(data, offsets, lens, n, chunk_len, np.uint8, gen_kind=A.GEN_EMPTY)
        assert e.value.code in (A.ANS_E_EXHAUSTED, A.ANS_E_MISMATCH), nbytes
    stream = torch.cuda.Stream()
    cap = gt.slot_capacity(chunk_len)
    slots = torch.zeros(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens_d = torch.full((nchunks,), cap + 64, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    gt.dev_decode(slots, None, cap, lens_d, n, chunk_len, out, sym_bytes, status, stream)
    assert gpu.status(status, stream) == A.ANS_E_LEN


def test_fast_kernel_errors(gpu):
    masses = A.c3_masses().copy()
    masses[7] = 0
    gt = A.GpuTable(gpu, A.Categorical(masses))
    syms = np.asarray(orc.gen_iid(masses, 3, 0, 64 * 4096), np.uint8)
    data, offsets, lens = gt.encode_chunks(syms, 4096)  # no symbol 7 was generated
    bad = syms.copy()
    bad[5 * 4096 + 17] = 7
    with pytest.raises(A.AnsError) as e:
        gt.encode_chunks(bad, 4096)
    assert e.value.code == A.ANS_E_ZERO_MASS
    gt2 = A.GpuTable(gpu, A.Categorical(masses[:200]))
    s2 = np.minimum(syms, 150).astype(np.uint8)
    s2[s2 == 7] = 8
    s2[3 * 4096 + 5] = 230  # out of range for a 200-symbol table
    with pytest.raises(A.AnsError) as e:
        gt2.encode_chunks(s2, 4096)
    assert e.value.code == A.ANS_E_SYMBOL


# ---------------------------------------------------------------- synthetic generator
def test_gen_iid_matches_oracle(gpu):
    torch = pytest.importorskip("torch")
    masses = A.c3_masses()
    gt = A.GpuTable(gpu, A.Categorical(masses))
    n, start = 1 << 20, 12345
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        gt.dev_gen_iid(1, start, n, d, 1, stream)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), orc.gen_iid(masses, 1, start, n).astype(np.uint8))


# ---------------------------------------------------------------- full-size configs (device-resident)
def _oracle_slices(masses, seed, n, chunk_len, nslices=64, start=0):
    """The oracle's streams of the whole workload, chunk-parallel on the host cores: contiguous
    chunk ranges (slices), each generated and encoded on its own thread (ctypes releases the
    GIL).  Returns [(c0, c1)], the lens of every chunk, and per slice the sha256 of its dense
    bytes."""
    from concurrent.futures import ThreadPoolExecutor
    import os
    nchunks = -(-n // chunk_len)
    per = -(-nchunks // nslices)
    bounds = [(c0, min(nchunks, c0 + per)) for c0 in range(0, nchunks, per)]

    def work(b):
        a, e = b[0] * chunk_len, min(n, b[1] * chunk_len)
        syms = orc.gen_iid(masses, seed, start + a, e - a)
        d, _, ln = orc.encode_chunks(masses, syms, chunk_len)
        return ln, hashlib.sha256(d.tobytes()).hexdigest()

    with ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1))) as ex:  # a GPU box's CPU share is 16
        res = list(ex.map(work, bounds))
    return bounds, np.concatenate([r[0] for r in res]).astype(np.int64), [r[1] for r in res]


def _device_roundtrip(gpu, masses, n, chunk_len, sym_bytes, seed, start=0):
    """Device-resident encode + decode of the whole workload (symbols [start, start + n) of the
    global array: one bench rank's shard); EVERY chunk's length and the bytes of the whole
    compacted stream (sha256 per slice of chunks) must equal the oracle's (src/ans.rs:255-260),
    and decode must be lossless."""
    torch = pytest.importorskip("torch")
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[sym_bytes]
    gt = A.GpuTable(gpu, A.Categorical(masses))
    stream = torch.cuda.Stream()  # a real stream: torch's default stream handle is NULL
    torch.cuda.set_stream(stream)
    nchunks = -(-n // chunk_len)
    cap = gt.slot_capacity(chunk_len)
    syms = torch.empty(n, dtype=dt, device="cuda")
    gt.dev_gen_iid(seed, start, n, syms, sym_bytes, stream)
    slots = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    gt.dev_encode(syms, sym_bytes, n, chunk_len, slots, cap, lens, status, stream)
    out = torch.empty_like(syms)
    gt.dev_decode(slots, None, cap, lens, n, chunk_len, out, sym_bytes, status, stream)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, syms), "lossless round trip"
    del out
    # the dense container (the wire format) of every chunk, built on the device
    # (ans_dev_encode_dense: encode + length scan + packing) and decoded in place
    l64 = lens.to(torch.int64)
    offs = torch.empty(A.dense_offsets_entries(nchunks), dtype=torch.int64, device="cuda")
    lens2 = torch.zeros_like(lens)
    dense = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
    gt.dev_encode_dense(syms, sym_bytes, n, chunk_len, slots, cap, lens2, offs, dense, status, stream)
    del slots
    assert torch.equal(lens2, lens), "dense encode: the same stream lengths"
    assert torch.equal(offs[:nchunks], torch.cumsum(l64, 0) - l64), "exclusive scan of the lengths"
    total = int(offs[nchunks].item())
    assert total == int(l64.sum().item())
    out = torch.empty_like(syms)
    gt.dev_decode(dense, offs, cap, lens, n, chunk_len, out, sym_bytes, status, stream)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, syms), "lossless round trip from the dense container"
    del out
    torch.cuda.synchronize()
    torch.cuda.set_stream(torch.cuda.default_stream())
    lens_h = l64.cpu().numpy()
    offs_h = offs[:nchunks].cpu().numpy()
    dense_h = dense[:total].cpu().numpy()
    del dense
    # the device generator is the oracle's (spot check; the streams below depend on all of it)
    ref = orc.gen_iid(masses, seed, start + n - 4096, 4096)
    assert np.array_equal(syms[n - 4096:].cpu().numpy().astype(np.int64) & ((1 << (8 * sym_bytes)) - 1), ref)
    bounds, olens, ohash = _oracle_slices(masses, seed, n, chunk_len, start=start)
    assert np.array_equal(lens_h, olens), "every chunk's stream length"
    for (c0, c1), h in zip(bounds, ohash):
        a = int(offs_h[c0])
        e = int(offs_h[c1]) if c1 < nchunks else total
        assert hashlib.sha256(dense_h[a:e].tobytes()).hexdigest() == h, f"chunks [{c0}, {c1})"
    return total


def test_c3_one_gib_u8_round_trip(gpu):
    # 2^30 u8 symbols, 256-symbol table (norm 139,224,331), chunk 4096;
    # all 262,144 chunks byte-compared against the oracle
    total = _device_roundtrip(gpu, A.c3_masses(), 1 << 30, 4096, 1, 1)
    bps = total / (1 << 30)
    assert 0.95 < bps < 0.99  # H = 7.738 bits -> ~0.967 B/symbol plus per-chunk flush


def test_c3_pow2_norm_bit_exact(gpu):
    # SURVEY.md §8d secondary C3: the table quantised to norm 2^24 (bench.py --config c3p2)
    masses = A.c3_pow2_masses()
    assert int(masses.sum()) == 1 << 24 and int(masses.min()) >= 1
    syms = orc.gen_iid(masses, 1, 0, 300 * 4096 + 17)
    _roundtrip_vs_oracle(gpu, masses, syms, 4096, np.uint8)


def test_c4_all_shards_u16_round_trip(gpu):
    # SURVEY.md §8d C4 (65,536 symbols, norm 134,561,356, 2^32 u16 symbols over 8 GPUs): every one
    # of the eight 2^29-symbol shards the bench codes (rank r: global symbols [r 2^29, (r+1) 2^29)),
    # one after the other on this GPU, so all 1,048,576 chunks of the workload have their lengths
    # and bytes compared against the oracle (src/codec.rs:405-443 per chunk)
    torch = pytest.importorskip("torch")
    n, shards = 1 << 29, 8
    totals = []
    for r in range(shards):
        totals.append(_device_roundtrip(gpu, A.c4_masses(), n, 4096, 2, 2, start=r * n))
        torch.cuda.empty_cache()  # the shard's buffers are gone: keep the device footprint at one shard
        assert 1.9 < totals[-1] / n < 2.1, f"shard {r}"
    # the shards concatenate to the 1-GPU container of the whole 2^32-symbol array:
    # its size is the sum over shards, 2 B of symbols against ~1.97 B of stream per symbol
    assert len(totals) == shards and 1.9 < sum(totals) / (shards * n) < 2.1


def test_compact_packs_exact_bytes(gpu):
    """ans_dev_compact (16-B packing with byte-exact first/last blocks): streams of every length
    class (0, 1, 15, 16, 17, ..., a whole slot) at every destination alignment land byte-exact,
    and no byte outside a stream is written (the gaps keep their sentinel)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    cap, nchunks = 256, 600
    lens_h = rng.integers(0, cap + 1, nchunks).astype(np.int64)
    lens_h[:8] = [0, 1, 15, 16, 17, 31, 33, cap]
    gaps = rng.integers(0, 40, nchunks)
    offs_h = np.cumsum(gaps + np.concatenate([[0], lens_h[:-1]])).astype(np.int64)
    slots_h = rng.integers(0, 256, nchunks * cap, dtype=np.uint8)
    total = int(offs_h[-1] + lens_h[-1]) + 64
    want = np.full(total, 0xAB, np.uint8)
    for j in range(nchunks):
        want[offs_h[j]:offs_h[j] + lens_h[j]] = slots_h[j * cap:j * cap + lens_h[j]]
    slots = torch.from_numpy(slots_h).cuda()
    lens = torch.from_numpy(lens_h.astype(np.int32)).cuda()
    offs = torch.from_numpy(offs_h).cuda()
    dense = torch.full((total,), 0xAB, dtype=torch.uint8, device="cuda")
    gpu.compact(slots, cap, lens, offs, nchunks, dense)
    torch.cuda.synchronize()
    assert np.array_equal(dense.cpu().numpy(), want)


@pytest.mark.parametrize("sym_bytes", [1, 2])
def test_dense_and_slot_layouts_decode_alike(gpu, sym_bytes):
    """ans_dev_decode_chunks on the dense container (explicit offsets, streams at any alignment,
    read in place) and on the encoder's slot layout give the same symbols and status, also for
    a corrupt stream that reads below its start (zeros there, not the previous chunk's bytes)."""
    torch = pytest.importorskip("torch")
    dt = {1: torch.uint8, 2: torch.int16}[sym_bytes]
    masses = A.c3_masses()
    gt = A.GpuTable(gpu, A.Categorical(masses))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    try:
        n, L = 700 * 4096 + 333, 4096
        nchunks = -(-n // L)
        cap = gt.slot_capacity(L)
        syms = torch.empty(n, dtype=dt, device="cuda")
        gt.dev_gen_iid(9, 0, n, syms, sym_bytes, stream)
        slots = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
        lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        gt.dev_encode(syms, sym_bytes, n, L, slots, cap, lens, status, stream)
        offsets = torch.zeros(nchunks, dtype=torch.int64, device="cuda")
        offsets[1:] = torch.cumsum(lens.to(torch.int64), 0)[:-1]
        dense = torch.empty(int(lens.to(torch.int64).sum().item()) + 16, dtype=torch.uint8, device="cuda")
        gpu.compact(slots, cap, lens, offsets, nchunks, dense, stream)
        out_fast = torch.empty_like(syms)
        out_generic = torch.empty_like(syms)
        gt.dev_decode(slots, None, cap, lens, n, L, out_fast, sym_bytes, status, stream)
        gt.dev_decode(dense, offsets, 0, lens, n, L, out_generic, sym_bytes, status, stream)
        assert gpu.status(status, stream) == 0
        assert torch.equal(out_fast, syms) and torch.equal(out_generic, syms)
        # a corrupted stream is caught by both layouts
        j = 123
        slots[j * cap + 5] ^= 0x5A
        dense[int(offsets[j].item()) + 5] ^= 0x5A
        status.zero_()
        gt.dev_decode(slots, None, cap, lens, n, L, out_fast, sym_bytes, status, stream)
        st_fast = gpu.status(status, stream)
        status.zero_()
        gt.dev_decode(dense, offsets, 0, lens, n, L, out_generic, sym_bytes, status, stream)
        st_generic = gpu.status(status, stream)
        assert st_fast == st_generic == A.ANS_E_MISMATCH
        assert torch.equal(out_fast, out_generic)
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.default_stream())


# ---------------------------------------------------------------- host-buffer pipeline
@pytest.mark.parametrize("sym_bytes,batch_bytes,depth", [(1, 1 << 20, None), (2, 3 << 19, None), (1, 4096 * 7, None),
                                                        (1, 1 << 20, "2"), (2, 1 << 20, "8")])
def test_host_pipeline_many_batches(sym_bytes, batch_bytes, depth, monkeypatch):
    """ans_gpu_encode_chunks / ans_gpu_decode_chunks split the call into batches that
    overlap copies and kernels; the container must equal the oracle's whatever the batch size
    and the number of workspace slots (ANS_PIPE_DEPTH), including a ragged last chunk in the
    last batch."""
    if depth is not None:
        monkeypatch.setenv("ANS_PIPE_DEPTH", depth)
    g = A.Gpu(0)
    g.set_batch_bytes(batch_bytes)
    masses = A.c3_masses()
    gt = A.GpuTable(g, A.Categorical(masses))
    dtype = {1: np.uint8, 2: np.uint16}[sym_bytes]
    n, L = 1000 * 4096 + 777, 4096
    syms = orc.gen_iid(masses, 11, 0, n).astype(dtype)
    assert g.pipe_depth() == 0  # built by the first host-buffer call
    data, offsets, lens = gt.encode_chunks(syms, L)
    assert g.pipe_depth() == (6 if depth is None else int(depth))  # the slot count really in use
    odata, ooffsets, olens = orc.encode_chunks(masses, syms.astype(np.uint32), L)
    assert np.array_equal(lens, olens) and np.array_equal(offsets, ooffsets)
    assert data.tobytes() == odata.tobytes()
    back = gt.decode_chunks(data, offsets, lens, n, L, dtype)
    assert np.array_equal(back, syms)
    # the same context again (workspace reuse), and a size query with no output buffer
    data2, _, _ = gt.encode_chunks(syms, L)
    assert data2.tobytes() == odata.tobytes()
    total = A.u64(0)
    rc = A.lib().ans_gpu_encode_chunks(gt.h, A._np_ptr(syms), sym_bytes, n, L, None, 0, None, None,
                                       A.ctypes.byref(total))
    assert rc == 0 and total.value == len(odata)


def test_host_pipeline_errors_and_scattered_container():
    g = A.Gpu(0)
    g.set_batch_bytes(1 << 18)
    masses = A.c3_masses()
    gt = A.GpuTable(g, A.Categorical(masses))
    n, L = 300 * 4096, 4096
    syms = orc.gen_iid(masses, 5, 0, n).astype(np.uint8)
    data, offsets, lens = gt.encode_chunks(syms, L)
    # output buffer one byte short: ANS_E_LEN, with the exact total still reported
    out = np.empty(len(data) - 1, np.uint8)
    offs = np.zeros(len(lens), np.uint64)
    ls = np.zeros(len(lens), np.uint64)
    total = A.u64(0)
    rc = A.lib().ans_gpu_encode_chunks(gt.h, A._np_ptr(syms), 1, n, L, A._np_ptr(out), len(out), A._np_ptr(offs),
                                       A._np_ptr(ls), A.ctypes.byref(total))
    assert rc == A.ANS_E_LEN and total.value == len(data)
    # streams stored far apart and out of order: the whole-buffer path decodes them
    gap = 10_000
    order = np.arange(len(lens))[::-1]
    scattered = np.zeros(int(lens.sum()) + gap * len(lens), np.uint8)
    soff = np.zeros(len(lens), np.uint64)
    pos = 0
    for j in order:
        soff[j] = pos
        scattered[pos:pos + int(lens[j])] = data[int(offsets[j]):int(offsets[j] + lens[j])]
        pos += int(lens[j]) + gap
    back = gt.decode_chunks(scattered, soff, lens, n, L, np.uint8)
    assert np.array_equal(back, syms)
    # a corrupted stream in a middle batch is reported
    bad = data.copy()
    bad[int(offsets[150]) + 3] ^= 0x33
    with pytest.raises(A.AnsError) as e:
        gt.decode_chunks(bad, offsets, lens, n, L, np.uint8)
    assert e.value.code == A.ANS_E_MISMATCH


@pytest.mark.parametrize("engine", ["runtime", "kernel"])
@pytest.mark.parametrize("sym_bytes,batch_bytes,skew", [(1, 1 << 20, 0), (2, 3 << 19, 0), (1, 4096 * 7, 3),
                                                       (2, 1 << 20, 5)])
def test_host_pipeline_page_locked(sym_bytes, batch_bytes, skew, engine, monkeypatch):
    """Page-locked (ans_host_alloc) buffers: asynchronous runtime copies (default), or with
    ANS_PIPE_COPY=kernel the device-driven path (copy kernels over PCIe, the container offset
    carried on the device).  `skew` shifts every buffer off 16-byte alignment."""
    monkeypatch.setenv("ANS_PIPE_COPY", engine)
    g = A.Gpu(0)
    g.set_batch_bytes(batch_bytes)
    masses = A.c3_masses()
    gt = A.GpuTable(g, A.Categorical(masses))
    dtype = {1: np.uint8, 2: np.uint16}[sym_bytes]
    n, L = 900 * 4096 + 1001, 4096
    ref = orc.gen_iid(masses, 13, 0, n).astype(dtype)
    syms = A.pinned_empty(n + skew, dtype)[skew:]
    syms[:] = ref
    nchunks = -(-n // L)
    cap = nchunks * gt.slot_capacity(L)
    out = A.pinned_empty(cap + skew, np.uint8)[skew:]
    offsets = np.zeros(nchunks, np.uint64)
    lens = np.zeros(nchunks, np.uint64)
    total = A.u64(0)
    A._check(A.lib().ans_gpu_encode_chunks(gt.h, A._np_ptr(syms), sym_bytes, n, L, A._np_ptr(out), cap,
                                           A._np_ptr(offsets), A._np_ptr(lens), A.ctypes.byref(total)), "encode")
    odata, ooffsets, olens = orc.encode_chunks(masses, ref.astype(np.uint32), L)
    assert total.value == len(odata)
    assert np.array_equal(lens, olens) and np.array_equal(offsets, ooffsets)
    assert out[:total.value].tobytes() == odata.tobytes()
    back = A.pinned_empty(n + skew, dtype)[skew:]
    A._check(A.lib().ans_gpu_decode_chunks(gt.h, A._np_ptr(out), total.value, A._np_ptr(offsets), A._np_ptr(lens),
                                           n, L, A.GEN_ZEROS, A._np_ptr(back), sym_bytes), "decode")
    assert np.array_equal(back, ref)
    # a too-small page-locked output: ANS_E_LEN with the exact total
    rc = A.lib().ans_gpu_encode_chunks(gt.h, A._np_ptr(syms), sym_bytes, n, L, A._np_ptr(out), total.value - 1,
                                       A._np_ptr(offsets), A._np_ptr(lens), A.ctypes.byref(total))
    assert rc == A.ANS_E_LEN and total.value == len(odata)
    # corruption in a middle batch is reported through the mapped path too
    out[int(ooffsets[nchunks // 2]) + 2] ^= 0x41
    rc = A.lib().ans_gpu_decode_chunks(gt.h, A._np_ptr(out), len(odata), A._np_ptr(offsets), A._np_ptr(lens),
                                       n, L, A.GEN_ZEROS, A._np_ptr(back), sym_bytes)
    assert rc == A.ANS_E_MISMATCH


# ---------------------------------------------------------------- Codec::samples in bulk
@pytest.mark.parametrize("which", ["c3", "multiset", "tiny_norm", "big_norm", "c4"])
def test_gpu_samples_match_host_and_oracle(gpu, which, multiset_masses):
    """Chunk c of ans_gpu_sample_iid = IID::new(codec, len).sample(seed + c) (src/ans.rs:42-44):
    the same symbols as the host coder and the C oracle (both Message::random, restated PCG)."""
    rng = np.random.default_rng(17)
    masses = {
        "c3": A.c3_masses(),
        "multiset": multiset_masses,
        "tiny_norm": np.asarray([3, 0, 5, 1, 7], np.uint64),
        "big_norm": rng.integers(1 << 22, 1 << 24, 300).astype(np.uint64),
        "c4": A.c4_masses(),
    }[which]
    cat = A.Categorical(masses)
    gt = A.GpuTable(gpu, cat)
    n, L, seed = 5000 * 7 + 3, 5000, 1234
    dtype = np.uint16 if len(masses) > 256 else np.uint8
    got = gt.sample_chunks(seed, n, L, dtype)
    ocat = orc.Categorical(masses)
    for c in range(-(-n // L)):
        ln = min(L, n - c * L)
        want = ocat.pop_iid(orc.Message.random(seed + c), ln)
        assert np.array_equal(got[c * L: c * L + ln], want.astype(dtype)), c
        if c < 2:
            assert A.IID(cat, ln).sample(seed + c) == [int(v) for v in want]
    if which == "c3":  # frequencies follow the masses (loose chi-square)
        big = gt.sample_chunks(99, 1 << 22, 4096, np.uint8)
        cnt = np.bincount(big, minlength=256).astype(np.float64)
        exp = masses.astype(np.float64) / masses.sum() * len(big)
        assert ((cnt - exp) ** 2 / exp).sum() < 400  # 255 dof


# ---------------------------------------------------------------- renorm step, adversarial
def _renorm_ref(head, window, L):
    """renorm_up (src/ans.rs:239-243): pull bytes (the window's top byte first) while head < L."""
    k = 0
    while head < L:
        head = ((head << 8) | ((window >> (24 - 8 * k)) & 0xFF)) & ((1 << 64) - 1)
        k += 1
    return head, k


@pytest.mark.parametrize("norm", [139_224_331, 268_434_941, (1 << 16) + 1, (1 << 31) - 1, 1 << 24, 3 * 5 ** 11])
def test_fast_renorm_exact_in_the_rare_window(gpu, norm):
    """The decoders take js = clz(head)/8 bytes unless X >> 8 already reaches L, which needs X in
    a window of width 2^56 mod norm (renorm_up's voted exact path): heads built to land there,
    mixed in the same waves with ordinary heads."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(norm % 1000)
    K = (1 << 56) // norm
    L = norm * K
    heads, wins = [], []
    for i in range(4096):
        w = int(rng.integers(0, 1 << 32))
        kind = i % 4
        if kind == 0:  # ordinary head after a pop, below L
            h = int(rng.integers(1 << 24, L))
        else:  # js = kind bytes, and X >> 8 inside [L, 2^56) or just below L
            js = kind
            lo = -(-(L - ((1 << (8 * (js - 1))) - 1)) // (1 << (8 * (js - 1))))  # head << 8(js-1) | ones >= L
            hi = 1 << (64 - 8 * js)
            h = int(rng.integers(max(lo - 3, 1 << 24), hi)) if hi > lo else int(rng.integers(1 << 24, hi))
            if rng.random() < 0.5:
                w = (1 << 32) - 1 - int(rng.integers(0, 256))  # top bytes near 0xFF: X >> 8 at the edge
        heads.append(min(h, (1 << 64) - 1))
        wins.append(w)
    d_h = torch.tensor(np.asarray(heads, np.uint64).view(np.int64), device="cuda")
    d_w = torch.tensor(np.asarray(wins, np.uint32).view(np.int32), device="cuda")
    o_h = torch.empty_like(d_h)
    o_k = torch.empty_like(d_w)
    A._check(A.lib().ans_dev_check_renorm(gpu.h, d_h.data_ptr(), d_w.data_ptr(), L, len(heads), o_h.data_ptr(),
                                          o_k.data_ptr(), None), "check_renorm")
    torch.cuda.synchronize()
    gh = o_h.cpu().numpy().view(np.uint64)
    gk = o_k.cpu().numpy().view(np.uint32)
    rare = 0
    for i, (h, w) in enumerate(zip(heads, wins)):
        eh, ek = _renorm_ref(h, w, L)
        assert (int(gh[i]), int(gk[i])) == (eh, ek), (i, hex(h), hex(w))
        js = min((64 - h.bit_length()) // 8, 4)
        rare += ek == js - 1 and js > 0
    if (1 << 56) - L > 0:
        assert rare > 100  # the exact path was exercised


# ---------------------------------------------------------------- table-shape boundaries
def _tables_at_the_boundaries():
    rng = np.random.default_rng(23)

    def spread(nsym, norm):  # nsym positive masses summing exactly to norm (distinct cut points)
        cuts = np.zeros(0, np.int64)
        while len(cuts) < nsym - 1:
            cuts = np.unique(np.concatenate([cuts, rng.integers(1, norm, 2 * nsym, dtype=np.int64)]))
        cuts = np.sort(rng.permutation(cuts)[:nsym - 1])
        return np.diff(np.concatenate([[0], cuts, [norm]])).astype(np.uint64)

    return {
        "norm_2^16": spread(256, 1 << 16),             # bottom of the fast range
        "norm_2^16-1": spread(256, (1 << 16) - 1),     # just below: generic kernels
        "norm_2^31": spread(256, 1 << 31),             # top of the fast range, L = 2^56
        "norm_2^31+1": spread(256, (1 << 31) + 1),     # just above: generic kernels
        "norm_2^32-1": spread(97, (1 << 32) - 1),      # largest norm the GPU takes
        "one_symbol": np.asarray([1 << 20], np.uint64),  # p = norm: nothing is ever emitted
        "kmax_4": np.concatenate([[1, 1, 2], spread(200, (1 << 31) - 4)]).astype(np.uint64),  # 4-byte pushes
        "pow2_norm_2^24": spread(256, 1 << 24),        # L = 2^56 exactly (empty renorm window)
    }


@pytest.mark.parametrize("name", ["norm_2^16", "norm_2^16-1", "norm_2^31", "norm_2^31+1", "norm_2^32-1", "one_symbol",
                                  "kmax_4", "pow2_norm_2^24"])
def test_boundary_tables_bit_exact(gpu, name):
    masses = _tables_at_the_boundaries()[name]
    rng = np.random.default_rng(len(name))
    nz = np.flatnonzero(masses)
    # uniform over the symbols, so the rare (tiny-mass) symbols are coded often
    syms = rng.choice(nz, size=520 * 4096 + 77).astype(np.uint32)
    _roundtrip_vs_oracle(gpu, masses, syms, 4096, np.uint8 if len(masses) <= 256 else np.uint16)


def test_rare_rows_whole_waves(gpu):
    """Rows that can emit kmax = 4 bytes per push (tiny masses: the one-compare renorm word
    ans_renorm.hpp enc_thr with k0 = 3; until r03f a wave-voted rare-row branch) under data made
    of them: chunks of only such symbols, half of them, and one in an otherwise common chunk.
    (CPU-checkable precondition: the table has kmax 4 and those rows hold at most 2^-10 of the
    mass, so common data rarely reaches them.)"""
    masses = _tables_at_the_boundaries()["kmax_4"]
    norm, K = int(masses.sum()), (1 << 56) // int(masses.sum())
    kmax_row = [max([j for j in range(1, 5) if (int(m) * K) << (8 * j) < 1 << 64], default=0) for m in masses]
    kmax = max(kmax_row)
    rare = [s for s, k in enumerate(kmax_row) if k == kmax]
    assert kmax == 4 and sum(int(masses[s]) for s in rare) << 10 <= norm
    rng = np.random.default_rng(41)
    L, nch = 4096, 192
    common = np.flatnonzero(np.asarray(kmax_row) < kmax)
    syms = rng.choice(common, size=(nch, L))
    syms[:64] = rng.choice(rare, size=(64, L))                      # waves of rare rows only
    half = rng.random((64, L)) < 0.5
    syms[64:128][half] = rng.choice(rare, size=int(half.sum()))
    syms[128:, 1000] = rare[0]                                      # one lane-step each
    _roundtrip_vs_oracle(gpu, masses, syms.reshape(-1).astype(np.uint32), L, np.uint8)


# ---------------------------------------------------------------- variable-length chunks
@pytest.mark.parametrize("which", ["c3", "multiset", "tiny_norm", "c4"])
def test_var_chunks_bit_exact(gpu, which, multiset_masses):
    """Chunk c = syms[starts[c]:starts[c+1]] (empty, one-symbol and long chunks mixed): each
    stream is the reference message of that slice alone (one oracle message per chunk).
    The large-alphabet tables (multiset: 1,024 symbols; c4) take the staged fast kernels."""
    rng = np.random.default_rng(31)
    masses = {"c3": A.c3_masses(), "multiset": multiset_masses,
              "tiny_norm": np.asarray([3, 0, 5, 1, 7], np.uint64), "c4": A.c4_masses()}[which]
    sizes = np.concatenate([[0, 1, 0, 7], rng.integers(0, 3000, 300), [20000, 0]]).astype(np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    n = int(starts[-1])
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    syms = rng.choice(nz, size=n, p=p / p.sum()).astype(np.uint32)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    dtype = np.uint16 if len(masses) > 256 else np.uint8
    data, offsets, lens = gt.encode_var_chunks(syms.astype(dtype), starts)
    for c in range(len(sizes)):
        a, b = int(starts[c]), int(starts[c + 1])
        od, _, ol = orc.encode_chunks(masses, syms[a:b], max(b - a, 1))
        want = od.tobytes() if b > a else bytes(orc.Message.zeros().flatten())
        got = data[int(offsets[c]):int(offsets[c] + lens[c])].tobytes()
        assert got == want, c
    back = gt.decode_var_chunks(data, offsets, lens, starts, dtype)
    assert np.array_equal(back, syms.astype(dtype))


@pytest.mark.parametrize("which,layout", [("c3", "mixed"), ("c4", "mixed"), ("multiset", "mixed"),
                                          ("c3", "one_long")])
def test_var_chunks_device_api_bit_exact(gpu, which, layout, multiset_masses):
    """ans_dev_encode_var_chunks_ex / ans_dev_decode_var_chunks_ex with device-resident starts:
    the library finds the longest chunk on the device and stages the chunks for the fast
    kernels (mixed lengths), or keeps the generic kernels when the padded layout would exceed
    its budget (one long chunk among a thousand empty ones).  Either way every slot holds the
    host API's (= the oracle's) stream of its chunk and decoding is lossless."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(47)
    masses = {"c3": A.c3_masses(), "multiset": multiset_masses, "c4": A.c4_masses()}[which]
    if layout == "mixed":
        sizes = np.concatenate([[0, 1, 0, 7], rng.integers(0, 3000, 300), [20000, 0]]).astype(np.uint64)
    else:
        sizes = np.concatenate([np.zeros(1000, np.uint64), [200_000], [5]]).astype(np.uint64)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    n, nchunks = int(starts[-1]), len(sizes)
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    syms = rng.choice(nz, size=n, p=p / p.sum()).astype(np.uint32)
    dtype, w = (np.uint16, 2) if len(masses) > 256 else (np.uint8, 1)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    ref, roffs, rlens = gt.encode_var_chunks(syms.astype(dtype), starts)
    cap = gt.slot_capacity(int(sizes.max()))
    stream = torch.cuda.Stream()
    tdt = torch.uint8 if w == 1 else torch.int16
    d_syms = torch.from_numpy(syms.astype(dtype).view(np.int16) if w == 2 else syms.astype(np.uint8)).to("cuda")
    d_starts = torch.from_numpy(starts.view(np.int64)).to("cuda")
    slots = torch.zeros(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = stream.cuda_stream
    A._check(A.lib().ans_dev_encode_var_chunks_ex(gt.h, d_syms.data_ptr(), w, nchunks, d_starts.data_ptr(), A.GEN_ZEROS,
                                                  0, slots.data_ptr(), cap, lens.data_ptr(), status.data_ptr(), s))
    out = torch.zeros(max(n, 1), dtype=tdt, device="cuda")
    A._check(A.lib().ans_dev_decode_var_chunks_ex(gt.h, slots.data_ptr(), None, cap, lens.data_ptr(), nchunks,
                                                  d_starts.data_ptr(), A.GEN_ZEROS, 0, out.data_ptr(), w,
                                                  status.data_ptr(), s))
    assert gpu.status(status, stream) == 0
    lens_h = lens.cpu().numpy().astype(np.uint64)
    assert np.array_equal(lens_h, rlens)
    slots_h = slots.cpu().numpy()
    for c in range(nchunks):
        got = slots_h[c * cap:c * cap + int(lens_h[c])].tobytes()
        assert got == ref[int(roffs[c]):int(roffs[c] + rlens[c])].tobytes(), c
    back = out[:n].cpu().numpy().view(dtype) if w == 2 else out[:n].cpu().numpy()
    assert np.array_equal(back, syms.astype(dtype))


# ---------------------------------------------------------------- large alphabets (ans_wide.hpp)
def _wide_table(rng, nsym, lo, hi, ones=0, zeros=0, crowd=0):
    masses = rng.integers(lo, hi, size=nsym, dtype=np.int64)
    if ones:  # mass-1 symbols: pushes of up to four bytes (kmax 4)
        masses[rng.choice(nsym, ones, replace=False)] = 1
    if crowd:  # runs of tiny masses: many cdf boundaries in one bucket (the voted scans)
        for start in rng.choice(nsym - 64, crowd, replace=False):
            masses[start:start + 40] = rng.integers(1, 4, 40)
    if zeros:
        masses[rng.choice(nsym, zeros, replace=False)] = 0
    return masses.astype(np.uint64)


@pytest.mark.parametrize("nsym,lo,hi,ones,zeros,crowd,chunk_len,n,compact,packed,shift", [
    (65536, 1, 1 << 12, 0, 0, 0, 4096, 600 * 4096 + 77, True, True, True),   # C4's shape, ragged tail
    (65536, 1, 1 << 12, 300, 500, 20, 4096, 520 * 4096, True, True, True),  # kmax 4, zero masses, crowded buckets
    (3000, 1 << 10, 1 << 13, 10, 0, 5, 64, 1200 * 64, True, False, False),   # small chunks (one 128-B group)
    (40000, 1, 1 << 16, 0, 0, 0, 2048, 600 * 2048, False, False, False),    # prefix and global parts both
                                                                            # large; offsets past u16
    (40000, 1, 5000, 0, 0, 0, 4096, 300 * 4096, None, True, False),         # packed, masses past the shift table
    (50000, 1, 1 << 12, 2000, 0, 0, 1024, 900 * 1024, None, True, True),    # shift table, many unit masses
])
def test_wide_kernels_bit_exact(gpu, nsym, lo, hi, ones, zeros, crowd, chunk_len, n, compact, packed, shift):
    """The large-alphabet kernels (k_encode_w: cdf-pair rows from the LDS prefix or global
    memory, 1/p by v_rcp_f64 + Newton, the renorm by bit lengths or by the per-mass shift byte;
    k_decode_w: LDS-prefix icdf + global buckets) against the oracle, symbols drawn from the
    table so both table parts and the scans are hit."""
    rng = np.random.default_rng(nsym + n)
    masses = _wide_table(rng, nsym, lo, hi, ones, zeros, crowd)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    assert gt.paths() & A.ANS_PATH_ENC_WIDE and gt.decode_kernel(2) == "wide"
    if compact is not None:
        assert bool(gt.paths() & A.ANS_PATH_DEC_COMPACT) == compact
    assert bool(gt.paths() & A.ANS_PATH_ENC_PACKED) == packed
    assert bool(gt.paths() & A.ANS_PATH_ENC_SHIFT) == shift
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    # half the symbols by probability, half uniform over the non-zero ones (tiny masses too)
    syms = np.where(rng.random(n) < 0.5, rng.choice(nz, size=n, p=p / p.sum()), rng.choice(nz, size=n))
    for dtype in (np.uint16, np.uint32):
        _roundtrip_vs_oracle(gpu, masses, syms.astype(np.uint32), chunk_len, dtype)


@pytest.mark.parametrize("table,chunk_len,n", [("c4", 1563, 300 * 1563 + 77), ("c4", 1, 500), ("c4", 63, 64 * 63),
                                               ("c4", 4100, 70 * 4100), ("c3", 1000, 600 * 1000 + 5),
                                               ("c3", 7, 3000), ("bernoulli", 333, 2000 * 333)])
def test_staged_ragged_chunks_bit_exact(gpu, table, chunk_len, n):
    """Chunk lengths whose bytes are no multiple of the fast kernels' 128-B groups (C2's 1,563
    u16 symbols) take the staged kernels (k_encode_w / k_decode_w, or the LDS-row k_encode /
    k_decode, with kVar), dense and slot layouts alike."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(chunk_len)
    masses = {"c4": A.c4_masses(), "c3": A.c3_masses(),
              "bernoulli": np.asarray([(1 << 28) - 26843, 26843], np.uint64)}[table]
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    syms = rng.choice(nz, size=n, p=p / p.sum()).astype(np.uint16)
    _roundtrip_vs_oracle(gpu, masses, syms.astype(np.uint32), chunk_len, np.uint16)
    if len(masses) <= 256:
        _roundtrip_vs_oracle(gpu, masses, syms.astype(np.uint32), chunk_len, np.uint8)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    try:
        nch = -(-n // chunk_len)
        cap = gt.slot_capacity(chunk_len)
        d_syms = torch.from_numpy(syms.view(np.int16)).cuda()
        slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
        lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        gt.dev_encode(d_syms, 2, n, chunk_len, slots, cap, lens, status, stream)
        out = torch.empty_like(d_syms)
        gt.dev_decode(slots, None, cap, lens, n, chunk_len, out, 2, status, stream)
        assert gpu.status(status, stream) == 0
        assert torch.equal(out, d_syms)
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.default_stream())


def test_wide_kernel_errors(gpu):
    rng = np.random.default_rng(3)
    masses = _wide_table(rng, 5000, 1 << 10, 1 << 13)
    masses[1234] = 0
    gt = A.GpuTable(gpu, A.Categorical(masses))
    assert gt.paths() & A.ANS_PATH_ENC_WIDE
    syms = rng.integers(0, 5000, size=600 * 4096).astype(np.uint16)
    syms[syms == 1234] = 1235
    gt.encode_chunks(syms, 4096)
    bad = syms.copy()
    bad[77 * 4096 + 5] = 1234  # zero mass (src/ans.rs:98)
    with pytest.raises(A.AnsError) as e:
        gt.encode_chunks(bad, 4096)
    assert e.value.code == A.ANS_E_ZERO_MASS
    bad = syms.copy()
    bad[300 * 4096 + 4095] = 60000  # out of range for a 5000-symbol table (src/codec.rs:63)
    with pytest.raises(A.AnsError) as e:
        gt.encode_chunks(bad, 4096)
    assert e.value.code == A.ANS_E_SYMBOL


# ---------------------------------------------------------------- Message::random initial messages
def _roundtrip_random(gpu, masses, syms, chunk_len, dtype, seed):
    gt = A.GpuTable(gpu, A.Categorical(masses))
    s = np.asarray(syms).astype(dtype)
    data, offsets, lens = gt.encode_chunks(s, chunk_len, gen_kind=A.GEN_RANDOM, seed=seed)
    od, oo, ol = orc.encode_chunks(masses, np.asarray(syms, np.uint32), chunk_len, kind=orc.RANDOM, seed=seed)
    assert np.array_equal(lens, ol)
    assert data.tobytes() == od.tobytes()
    back = gt.decode_chunks(data, offsets, lens, len(s), chunk_len, dtype, gen_kind=A.GEN_RANDOM, seed=seed)
    assert np.array_equal(back, s)
    with pytest.raises(A.AnsError) as e:  # another seed's initial message is not where decoding ends
        gt.decode_chunks(data, offsets, lens, len(s), chunk_len, dtype, gen_kind=A.GEN_RANDOM, seed=seed + 1)
    assert e.value.code == A.ANS_E_MISMATCH
    return data


@pytest.mark.parametrize("size,chunks", [(1000, 1), (100000, 1), (100000, 64)])
def test_random_message_multiset_fixtures(gpu, size, chunks, multiset_masses, multiset_vectors):
    """The reference harness codes each fixture from Message::random(0) (src/multiset.rs:174,
    src/benchmark.rs:698-700): one chunk with seed 0 is exactly that message (C1 on the HIP
    path); 64 chunks give chunk c Message::random(c) (C2 layout)."""
    syms = multiset_vectors[size]
    chunk_len = -(-size // chunks)
    for dtype in (np.uint16, np.uint32):
        _roundtrip_random(gpu, multiset_masses, syms, chunk_len, dtype, 0)


@pytest.mark.parametrize("which", ["c3", "c4", "bernoulli", "c4_staged", "c3_staged"])
def test_random_message_fast_kernels(gpu, which):
    """Message::random(seed + c) on the fast kernels (LDS rows / wide tables, and their staged
    ragged-chunk forms), against the oracle."""
    chunk_len = 4096
    if which == "c3":
        masses, n, dtype = A.c3_masses(), 1100 * 4096 + 5, np.uint8
    elif which == "c4":
        masses, n, dtype = A.c4_masses(), 600 * 4096, np.uint16
    elif which == "c4_staged":
        masses, n, dtype, chunk_len = A.c4_masses(), 300 * 1563 + 11, np.uint16, 1563
    elif which == "c3_staged":
        masses, n, dtype, chunk_len = A.c3_masses(), 500 * 1000 + 3, np.uint8, 1000
    else:
        masses, n, dtype = np.array([(1 << 28) - 26843, 26843], np.uint64), 700 * 4096, np.uint8
    syms = orc.gen_iid(masses, 9, 0, n)
    _roundtrip_random(gpu, masses, syms, chunk_len, dtype, 12345)


@pytest.mark.parametrize("which", ["c3", "c4", "c3_long"])
def test_random_message_dense_container(gpu, which):
    """ans_dev_encode_dense_ex from Message::random(seed + c): the packed bytes equal the
    oracle's, and decoding the container in place returns the symbols (c3_long: 64-KiB
    streams, so the pack runs many passes of four 64-block rounds and carries across them)."""
    torch = pytest.importorskip("torch")
    seed, L = 4242, 4096
    if which == "c3":
        masses, n, sb = A.c3_masses(), 300 * 4096, 1
    elif which == "c4":
        masses, n, sb = A.c4_masses(), 200 * 4096, 2
    else:
        masses, n, sb, L = A.c3_masses(), 40 * 65536, 1, 65536
    gt = A.GpuTable(gpu, A.Categorical(masses))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    try:
        nch = n // L
        cap = gt.slot_capacity(L)
        syms = torch.empty(n, dtype=torch.uint8 if sb == 1 else torch.int16, device="cuda")
        gt.dev_gen_iid(5, 0, n, syms, sb, stream)
        slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
        lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
        offs = torch.empty(A.dense_offsets_entries(nch), dtype=torch.int64, device="cuda")
        dense = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        gt.dev_encode_dense(syms, sb, n, L, slots, cap, lens, offs, dense, status, stream,
                            gen_kind=A.GEN_RANDOM, seed=seed)
        out = torch.empty_like(syms)
        gt.dev_decode(dense, offs, cap, lens, n, L, out, sb, status, stream, gen_kind=A.GEN_RANDOM, seed=seed)
        assert gpu.status(status, stream) == 0
        assert torch.equal(out, syms)
        torch.cuda.synchronize()
        total = int(offs[nch].item())
        host = syms.cpu().numpy().view(np.uint8 if sb == 1 else np.uint16).astype(np.uint32)
        od, _, ol = orc.encode_chunks(masses, host, L, kind=orc.RANDOM, seed=seed)
        assert np.array_equal(lens.cpu().numpy().astype(np.int64), ol.astype(np.int64))
        assert dense[:total].cpu().numpy().tobytes() == od.tobytes()
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.default_stream())


def test_random_message_device_api(gpu):
    """ans_dev_*_chunks_ex: slot layout, device buffers, seed offsets per chunk."""
    torch = pytest.importorskip("torch")
    masses = A.c3_masses()
    gt = A.GpuTable(gpu, A.Categorical(masses))
    n, L, seed = 1 << 22, 4096, 777
    stream = torch.cuda.Stream()
    syms = torch.empty(n, dtype=torch.uint8, device="cuda")
    gt.dev_gen_iid(3, 0, n, syms, 1, stream)
    cap = gt.slot_capacity(L)
    slots = torch.empty((n // L) * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(n // L, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    gt.dev_encode(syms, 1, n, L, slots, cap, lens, status, stream, gen_kind=A.GEN_RANDOM, seed=seed)
    out = torch.empty_like(syms)
    gt.dev_decode(slots, None, cap, lens, n, L, out, 1, status, stream, gen_kind=A.GEN_RANDOM, seed=seed)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, syms)
    lh = lens.cpu().numpy()
    ref = orc.gen_iid(masses, 3, 0, n)
    od, oo, ol = orc.encode_chunks(masses, ref, L, kind=orc.RANDOM, seed=seed)
    assert np.array_equal(lh.astype(np.uint64), ol)
    sl = slots.cpu().numpy()
    for c in (0, 1, 511, 1023):
        assert sl[c * cap: c * cap + lh[c]].tobytes() == od[int(oo[c]):int(oo[c]) + int(ol[c])].tobytes()


def _wide_rerun_masses():
    """1,000 symbols (the wide decoder, ans_wide.hpp k_decode_w) with a few large masses."""
    rng = np.random.default_rng(5)
    m = rng.integers(1, 4097, 1000).astype(np.uint64)
    m[[3, 500, 998]] = [1 << 22, 3 << 21, 1 << 21]
    return m


def _norm255_masses():
    """40 masses summing to 255 (kNormSmall at norm <= 256: the 24-bit high-word product off)."""
    m = np.full(40, 6, np.int64)
    m[:15] += 1
    assert int(m.sum()) == 255
    return m.astype(np.uint64)


def _wide_small_masses():
    """1,000 symbols below 2^16 (the wide decoder's kNormSmall long division) with large masses."""
    rng = np.random.default_rng(6)
    m = rng.integers(1, 40, 1000).astype(np.uint64)
    m[[3, 500, 998]] = [9000, 6000, 5000]
    assert int(m.sum()) < (1 << 16)
    return m


@pytest.mark.parametrize("which", ["c3_u8", "wide_u16", "c3_small_u8", "norm255_u8", "wide_small_u16"])
def test_decoder_deferred_screen_reruns_the_unit(gpu, which):
    """The C3 decoder takes the renorm's one-byte-less screen once per unit (ans_fast.hpp
    k_decode kDefer) and re-runs a unit where a lane reached it; the large-alphabet decoder
    (ans_wide.hpp k_decode_w) screens every step.  Chunks whose first pop leaves the head at
    exactly L (inside the window [L, 2^56) where the clz rule pulls one byte too many) take
    that path; they sit in the same waves as ordinary chunks, and every chunk's symbols must
    equal the oracle's pops of the same stream (the crafted streams end in a mismatch status,
    which the ordinary ones must not share).  The kNormSmall tables (norm 32,749, norm 255, and
    1,000 symbols below 2^16 on the wide decoder) take the same re-run through their long-division
    quotient (ans_fast.hpp renorm_div_u's div_hi state)."""
    torch = pytest.importorskip("torch")
    masses = {"c3_u8": A.c3_masses, "wide_u16": _wide_rerun_masses, "c3_small_u8": A.c3_small_masses,
              "norm255_u8": _norm255_masses, "wide_small_u16": _wide_small_masses}[which]()
    sym_bytes = 1 if which.endswith("u8") else 2
    norm = int(masses.sum())
    K = (1 << 56) // norm
    L = norm * K
    assert L < (1 << 56)
    cum = np.concatenate([[0], np.cumsum(masses.astype(np.int64))])
    big = [s for s in range(len(masses)) if int(masses[s]) * 250 > norm]  # H = q norm + cf < 2^64
    chunk_len, nch = 4096, 512
    rng = np.random.default_rng(77)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    assert gt.decode_kernel(sym_bytes) == ("lds" if sym_bytes == 1 else "wide")
    cap = gt.slot_capacity(chunk_len)
    slots = np.zeros(nch * cap, np.uint8)
    lens = np.zeros(nch, np.uint32)
    want = np.zeros(nch * chunk_len, np.uint32)
    ocat = orc.Categorical(masses)
    crafted = []
    for c in range(nch):
        if c % 3 == 1:  # crafted: H such that the first pop of symbol s leaves head = L
            s = int(big[int(rng.integers(0, len(big)))])
            q, rr = divmod(L, int(masses[s]))
            H = norm * q + int(cum[s]) + rr
            assert L <= H < (1 << 64)
            data = orc.Message.unflatten(H.to_bytes(8, "little").rstrip(b"\0") or b"\0").flatten()
            m1 = orc.Message.unflatten(data)
            assert ocat.pop(m1) == s and m1.head == L  # the reference kept the head at L (no byte)
            want[c * chunk_len:(c + 1) * chunk_len] = ocat.pop_iid(orc.Message.unflatten(data), chunk_len)
            crafted.append(c)
        else:  # an ordinary chunk
            syms = orc.gen_iid(masses, 1000 + c, 0, chunk_len)
            m = orc.Message.zeros()
            ocat.push_iid(m, syms)
            data = m.flatten()
            want[c * chunk_len:(c + 1) * chunk_len] = syms
        assert len(data) <= cap
        slots[c * cap:c * cap + len(data)] = np.frombuffer(data, np.uint8)
        lens[c] = len(data)
    d_slots = torch.from_numpy(slots).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    dt = np.uint8 if sym_bytes == 1 else np.uint16
    out = torch.zeros(nch * chunk_len, dtype=torch.uint8 if sym_bytes == 1 else torch.int16, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    gt.dev_decode(d_slots, None, cap, d_lens, nch * chunk_len, chunk_len, out, sym_bytes, status)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(dt)
    for c in range(nch):
        assert np.array_equal(got[c * chunk_len:(c + 1) * chunk_len], want[c * chunk_len:(c + 1) * chunk_len].astype(dt)), c
    assert int(status.item()) == 1 << A.ANS_E_MISMATCH  # the crafted streams do not return to their start
