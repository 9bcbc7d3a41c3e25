"""GPU parity of the fast kernels for the codecs beside IID<Categorical> (ans_mfast.hpp, include/
ans_capi.h section 4b): Independent<Categorical> over <= 256-symbol tables in LDS, IID<Uniform>,
IID<LogUniform>.  Every chunk's bytes must equal the oracle's (oracle/ans_oracle.c orc_codec_*,
the restatement of src/codec.rs:13-49,366-403,561-611 and src/ans.rs:96-116,233-264), decode must
be lossless and end at the initial message, through the host-buffer and the device-resident
calls alike.  Includes constructed chunks that drive the bidirectional renorm (a push taking a
byte back, a pop handing one back, src/ans.rs:233-253), which random data reaches about once in
2^30 symbols."""
import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    return A.Gpu(0)


def _sample(rng, masses, n):
    nz = np.flatnonzero(masses)
    p = masses[nz].astype(np.float64)
    return rng.choice(nz, size=n, p=p / p.sum())


def _indep_case(rng, tables, n):
    tids = rng.integers(0, len(tables), size=n).astype(np.uint32)
    syms = np.zeros(n, np.uint64)
    for t, m in enumerate(tables):
        sel = tids == t
        syms[sel] = _sample(rng, m, int(sel.sum()))
    return tids, syms


def _check_indep(ts, tables, tids, syms, L, dtype, kind=A.GEN_ZEROS, seed=0):
    s = syms.astype(dtype)
    data, offsets, lens = ts.encode_chunks(tids, s, L, kind, seed)
    od, oo, ol = orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, syms, L, tables=tables, tids=tids, kind=kind, seed=seed)
    assert np.array_equal(lens, ol), "stream lengths"
    assert data.tobytes() == od.tobytes(), "stream bytes"
    back = ts.decode_chunks(tids, data, offsets, lens, L, dtype, kind, seed)
    assert np.array_equal(back, s), "lossless"
    return data, offsets, lens


def _fast_tables(rng):
    """Five 256-symbol tables in the fast range, as tools/codecs_bench.py codes them."""
    return [rng.integers(1, 1 << 16, size=256).astype(np.uint64) for _ in range(5)]


def _mixed_tables(rng):
    """Norms from 2^16 to 2^31, zero masses, small alphabets, a near-deterministic symbol."""
    t = [rng.integers(1, 1 << 20, size=256).astype(np.uint64),
         rng.integers(0, 1 << 12, size=17).astype(np.uint64),
         np.array([(1 << 16) - 3, 3], np.uint64),
         rng.integers(1 << 22, 1 << 23, size=200).astype(np.uint64),
         np.array([(1 << 31) - 1000, 999, 1], np.uint64)]
    t[1][0] = 1 << 16  # norm >= 2^16
    t[1][5] = 0
    return t


@pytest.mark.parametrize("lanes", [256, 1024])
@pytest.mark.parametrize("dtype,L", [(np.uint8, 4096), (np.uint8, 128), (np.uint16, 1024), (np.uint32, 32)])
def test_independent_fast_bit_exact(gpu, dtype, L, lanes):
    """Both kernel layouts (256-lane workgroups, or 1,024 sharing one LDS table image, which
    calls of at least 1,024 chunks per CU take by default) code the same bytes."""
    rng = np.random.default_rng(L + np.dtype(dtype).itemsize)
    tables = _fast_tables(rng)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    ts.lanes(lanes)
    assert ts.fast() == 1
    n = 37 * L + 29  # a ragged last chunk (exact kernel) after the fast chunks
    tids, syms = _indep_case(rng, tables, n)
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 9), (A.GEN_EMPTY, 0)]:
        _check_indep(ts, tables, tids, syms, L, dtype, kind, seed)


@pytest.mark.parametrize("dtype,L", [(np.uint8, 256), (np.uint16, 64), (np.uint32, 4096)])
def test_independent_fast_mixed_norms(gpu, dtype, L):
    rng = np.random.default_rng(100 + L)
    tables = _mixed_tables(rng)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    assert ts.fast() in (1, 2)
    n = 301 * L
    tids, syms = _indep_case(rng, tables, n)
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 4)]:
        _check_indep(ts, tables, tids, syms, L, dtype, kind, seed)


def _lean_edge_tables(rng):
    """Lean sets (masses < 2^24, kmax <= 3) at the ends of the nearest-rounded quotient's range
    (ans_mfast.hpp IndepModel::pop): norms just below 2^31, where q' = q - 1 and q' = q + 1 leave
    overlapping 32-bit remainders (the voted fix-up decides in 64 bits), and norms of exactly 2^20,
    where the estimate misses most often; crowded buckets (small masses) among them."""
    big = rng.integers(1 << 23, 1 << 24, size=256).astype(np.uint64)
    big = (big * ((1 << 31) - 7) // int(big.sum())).astype(np.uint64)
    big[0] += np.uint64((1 << 31) - 7 - int(big.sum()))
    crowd = np.concatenate([np.full(200, 64, np.int64), rng.integers(1 << 23, 1 << 24, size=56)])  # p K >= 2^32
    t20 = np.maximum(1, rng.integers(1, 1 << 13, size=256) * (1 << 20) // (1 << 20))
    t20 = np.maximum(1, t20 * (1 << 20) // int(t20.sum()))
    t20[int(np.argmax(t20))] += (1 << 20) - int(t20.sum())
    small20 = np.array([(1 << 20) - 5, 2, 3], np.uint64)
    return [big, crowd.astype(np.uint64), t20.astype(np.uint64), small20]


@pytest.mark.parametrize("lanes", [256, 1024])
@pytest.mark.parametrize("dtype,L", [(np.uint8, 4096), (np.uint16, 512)])
def test_independent_fast_lean_quotient_edges(gpu, dtype, L, lanes):
    rng = np.random.default_rng(500 + L)
    tables = _lean_edge_tables(rng)
    for m in tables:
        assert (1 << 20) <= int(m.sum()) < (1 << 31) and int(m.max()) < (1 << 24)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    ts.lanes(lanes)
    assert ts.fast() == 1
    n = 257 * L
    tids = rng.integers(0, len(tables), size=n).astype(np.uint32)
    syms = np.zeros(n, np.uint64)
    for t, m in enumerate(tables):  # half uniform over the symbols (rare rows, crowded buckets)
        sel = np.flatnonzero(tids == t)
        p = m.astype(np.float64) / float(m.sum())
        syms[sel] = np.where(rng.random(len(sel)) < 0.5, rng.choice(len(m), size=len(sel), p=p),
                             rng.choice(np.flatnonzero(m), size=len(sel)))
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 6)]:
        _check_indep(ts, tables, tids, syms, L, dtype, kind, seed)


def _small_norm_tables(rng):
    """Count-built tables below 2^16 (src/benchmark.rs:549-578): a dataset edge Bernoulli, label
    counts with an absent label, Bernoulli::new(1, 2) (src/param_codec.rs:273), a 256-symbol one."""
    return [np.array([31000, 3400], np.uint64), np.array([2395, 345, 593, 0, 23, 12, 2], np.uint64),
            np.array([1, 1], np.uint64), rng.integers(1, 200, size=256).astype(np.uint64),
            np.array([65000, 1, 1, 7], np.uint64)]


def _big_norm_tables(rng):
    """Norms in (2^31, 2^32), a mass above 2^31 among them."""
    t = [rng.integers(1 << 23, 1 << 24, size=256).astype(np.uint64),
         np.array([(1 << 31) + 12345, 1, 77, 1 << 30], np.uint64),
         np.array([(1 << 32) - 2, 1], np.uint64)]
    t[0] = (t[0] * ((1 << 32) - 99) // int(t[0].sum())).astype(np.uint64)
    return t


@pytest.mark.parametrize("lanes", [256, 1024])
@pytest.mark.parametrize("which", ["small", "big"])
@pytest.mark.parametrize("dtype,L", [(np.uint8, 4096), (np.uint8, 128), (np.uint16, 512)])
def test_independent_fast_norm_ranges(gpu, which, dtype, L, lanes):
    """Sets whose norms all lie below 2^16 (or all in (2^31, 2^32)) take the fast kernels with
    the long-division (64-bit-checked) quotient of ans_fast.hpp kNormSmall (kNormBig), in both
    workgroup layouts: 256 lanes (what dataset-sized calls take by default) and 1,024 lanes
    sharing one LDS image (the big set's decoder image does not fit 28 KiB: its decodes stay on
    256 lanes there)."""
    rng = np.random.default_rng(300 + L + len(which))
    tables = _small_norm_tables(rng) if which == "small" else _big_norm_tables(rng)
    for m in tables:
        assert (int(m.sum()) < 1 << 16) if which == "small" else ((1 << 31) < int(m.sum()) < (1 << 32))
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    ts.lanes(lanes)
    assert ts.fast() in (1, 2)
    n = 301 * L + 17
    tids = rng.integers(0, len(tables), size=n).astype(np.uint32)
    syms = np.zeros(n, np.uint64)
    for t, m in enumerate(tables):  # uniform over each table's symbols: the rare rows often
        sel = tids == t
        syms[sel] = rng.choice(np.flatnonzero(m), size=int(sel.sum()))
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 4), (A.GEN_EMPTY, 0)]:
        _check_indep(ts, tables, tids, syms, L, dtype, kind, seed)


def test_independent_exact_only_sets(gpu):
    """Sets the fast kernels decline stay bit-exact on the exact kernels: norms from two ranges in
    one set, and sixteen 256-symbol tables (16 x 8,224 B of encoder rows pass the LDS)."""
    rng = np.random.default_rng(77)
    mixed = [rng.integers(1, 1 << 16, size=256).astype(np.uint64), np.array([3, 5], np.uint64)]
    sixteen = [rng.integers(1, 1 << 16, size=256).astype(np.uint64) for _ in range(16)]
    fifteen = sixteen[:15]
    for tables, fast in [(mixed, 0), (sixteen, 0), (fifteen, 1)]:
        ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
        assert ts.fast() == fast, len(tables)
        tids, syms = _indep_case(rng, tables, 40 * 256)
        _check_indep(ts, tables, tids, syms, 256, np.uint8)


def _renorm_tables():
    """Tables whose pushes, in the order below, leave a head of 2^56 - 2^25 before a push with
    p K = 2^56 - 1, which must take a byte back (see the docstring of the test)."""
    return [np.array([1 << 15, 1 << 15], np.uint64),         # E: norm 2^16, p = 2^15
            np.array([1, (1 << 31) - 2], np.uint64),         # C: norm 2^31 - 1, p = 1 (K = 2^25)
            np.array([71755], np.uint64),                    # D: norm 71755 | 2^56 - 1: p K = 2^56 - 1
            np.array([1, (1 << 16) - 1], np.uint64),         # F: norm 2^16, p = 1: 2 bytes, head back to 2^56
            np.array([1, (1 << 24) - 1], np.uint64),         # G: norm 2^24, p = 1: 3 bytes, head back to 2^56
            np.arange(1, 257, dtype=np.uint64) * 97]         # A: an ordinary table for the rest


@pytest.mark.parametrize("dtype,L", [(np.uint8, 256), (np.uint16, 128)])
def test_independent_fast_bidirectional_renorm(gpu, dtype, L):
    """Chunk c ends with D, C, E and then a run of F / G pushes (pushed first: IID pushes the last
    position first).  From Message::zeros() the F / G pushes emit 2 or 3 bytes each and return
    the head to exactly 2^56; E's push (p / norm = 1/2) makes it 2^57 + 2^15; C's (p = 1,
    K = 2^25) emits 4 bytes and leaves norm_C * 2^25 = 2^56 - 2^25 < p K of D's single symbol
    (2^56 - 1): D's push takes the last byte back (src/ans.rs:239-243), and decoding C's pop hands
    it back (renorm_down, src/ans.rs:246-253).  The F / G runs vary per chunk, so the take-back
    lands at every byte offset of a dword and on both sides of a 64-B page boundary."""
    rng = np.random.default_rng(5)
    tables = _renorm_tables()
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    assert ts.fast() == 2  # D's row takes the voted exact renorm
    E, C, D, F, G, Atab = range(6)
    nchunks = 96
    tids = np.zeros(nchunks * L, np.uint32)
    syms = np.zeros(nchunks * L, np.uint64)
    for c in range(nchunks):
        a, b = c % 17, (c // 17) % 6  # 2a + 3b bytes before E, C, D
        run = [F] * a + [G] * b
        rng.shuffle(run)
        tail = [D, C, E] + run
        head = L - len(tail)
        tt = np.concatenate([np.full(head, Atab), np.array(tail)]).astype(np.uint32)
        ss = np.zeros(L, np.uint64)
        ss[:head] = _sample(rng, tables[Atab], head)
        ss[head + 2] = 1  # E's symbol 1 (p = 2^15, cdf 2^15); D, C, F, G: symbol 0
        tids[c * L:(c + 1) * L] = tt
        syms[c * L:(c + 1) * L] = ss
    _check_indep(ts, tables, tids, syms, L, dtype)
    # the same chunks in the device-resident calls, in slots and from the dense container
    torch = pytest.importorskip("torch")
    stream = torch.cuda.Stream()
    d_tids = torch.from_numpy(tids.astype(np.uint8)).cuda()
    d_syms = torch.from_numpy(syms.astype(dtype).view(np.uint8)).cuda()
    cap = ts.slot_capacity(L)
    slots = torch.zeros(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    w = np.dtype(dtype).itemsize
    ts.dev_encode(d_tids, d_syms, w, len(syms), L, slots, cap, lens, status, stream)
    out = torch.zeros_like(d_syms)
    ts.dev_decode(d_tids, slots, None, cap, lens, len(syms), L, out, w, status, stream)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, d_syms)
    od, oo, ol = orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, syms, L, tables=tables, tids=tids)
    h = slots.cpu().numpy().reshape(nchunks, cap)
    ln = lens.cpu().numpy()
    assert np.array_equal(ln, ol)
    for c in range(nchunks):
        assert h[c, :ln[c]].tobytes() == od[oo[c]:oo[c] + ol[c]].tobytes(), f"chunk {c}"


def test_independent_fast_device_api_dense(gpu):
    """ans_dev_independent_*: slots and the dense container (decoded in place) equal the oracle."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(8)
    tables = _fast_tables(rng)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    L, nchunks = 1024, 300
    n = L * nchunks
    tids, syms = _indep_case(rng, tables, n)
    stream = torch.cuda.Stream()
    d_tids = torch.from_numpy(tids.astype(np.uint8)).cuda()
    d_syms = torch.from_numpy(syms.astype(np.uint8)).cuda()
    cap = ts.slot_capacity(L)
    slots = torch.zeros(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    ts.dev_encode(d_tids, d_syms, 1, n, L, slots, cap, lens, status, stream, A.GEN_RANDOM, 3)
    od, oo, ol = orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, syms, L, tables=tables, tids=tids, kind=A.GEN_RANDOM,
                                         seed=3)
    ln = lens.cpu().numpy().astype(np.uint64)
    assert np.array_equal(ln, ol)
    dense = np.concatenate([slots.cpu().numpy().reshape(nchunks, cap)[c, :ln[c]] for c in range(nchunks)])
    assert dense.tobytes() == od.tobytes()
    d_dense = torch.from_numpy(dense).cuda()
    d_offs = torch.from_numpy(oo.astype(np.int64)).cuda()
    out = torch.zeros_like(d_syms)
    ts.dev_decode(d_tids, d_dense, d_offs, cap, lens, n, L, out, 1, status, stream, A.GEN_RANDOM, 3)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, d_syms)


@pytest.mark.parametrize("offsets", [(1, 0, 0), (0, 3, 0), (0, 0, 8), (5, 7, 4)])
def test_independent_misaligned_device_buffers(gpu, offsets):
    """ans_dev_independent_*: the fast kernels move symbols, table ids and slot pages with 16-B
    vector accesses; views offset from 16-B alignment (symbols, ids, slots) take the exact kernels
    and code the same bytes."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(9)
    tables = _fast_tables(rng)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    L, nchunks = 1024, 64
    n = L * nchunks
    tids, syms = _indep_case(rng, tables, n)
    os_, ot, ob = offsets
    stream = torch.cuda.Stream()
    d_syms = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")[os_:os_ + n]
    d_syms.copy_(torch.from_numpy(syms.astype(np.uint8)))
    d_tids = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")[ot:ot + n]
    d_tids.copy_(torch.from_numpy(tids.astype(np.uint8)))
    cap = ts.slot_capacity(L)
    slots = torch.zeros(nchunks * cap + 16, dtype=torch.uint8, device="cuda")[ob:ob + nchunks * cap]
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    ts.dev_encode(d_tids, d_syms, 1, n, L, slots, cap, lens, status, stream)
    assert gpu.status(status, stream) == 0
    od, oo, ol = orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, syms, L, tables=tables, tids=tids)
    ln = lens.cpu().numpy().astype(np.uint64)
    assert np.array_equal(ln, ol)
    sl = slots.cpu().numpy().reshape(nchunks, cap)
    assert np.concatenate([sl[c, :ln[c]] for c in range(nchunks)]).tobytes() == od.tobytes()
    out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")[os_:os_ + n]
    ts.dev_decode(d_tids, slots, None, cap, lens, n, L, out, 1, status, stream)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, d_syms)


def test_independent_fast_errors_and_corruption(gpu):
    rng = np.random.default_rng(2)
    tables = _mixed_tables(rng)
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    L = 256
    tids, syms = _indep_case(rng, tables, 40 * L)
    bad = syms.copy()
    bad[np.flatnonzero(tids == 1)[3]] = 17  # out of range for the 17-symbol table (src/codec.rs:63)
    with pytest.raises(A.AnsError) as e:
        ts.encode_chunks(tids, bad.astype(np.uint8), L)
    assert e.value.code == A.ANS_E_SYMBOL
    bad = syms.copy()
    bad[np.flatnonzero(tids == 1)[3]] = 5  # zero mass (src/ans.rs:98)
    with pytest.raises(A.AnsError) as e:
        ts.encode_chunks(tids, bad.astype(np.uint8), L)
    assert e.value.code == A.ANS_E_ZERO_MASS
    data, offsets, lens = ts.encode_chunks(tids, syms.astype(np.uint8), L)
    for pos in (0, int(offsets[7]) + 3, int(offsets[20]) + int(lens[20]) - 1):
        d2 = data.copy()
        d2[pos] ^= 0x5A
        try:
            back = ts.decode_chunks(tids, d2, offsets, lens, L, np.uint8)
        except A.AnsError as err:
            assert err.code in (A.ANS_E_MISMATCH, A.ANS_E_EXHAUSTED)
        else:
            raise AssertionError(f"corrupt byte {pos} decoded without an error: {np.count_nonzero(back != syms)}")


@pytest.mark.parametrize("size", [1, 2, 3, 1000, (1 << 16) + 1, (1 << 28) - 57, 1 << 40, (1 << 40) + 7, 1 << 46])
@pytest.mark.parametrize("dtype,L", [(np.uint64, 4096), (np.uint64, 16), (np.uint32, 128), (np.uint8, 256)])
def test_uniform_fast_bit_exact(gpu, size, dtype, L):
    rng = np.random.default_rng(size % 977 + L)
    hi = min(size, 1 << (8 * np.dtype(dtype).itemsize))
    n = 41 * L + 5
    syms = rng.integers(0, hi, size=n, dtype=np.uint64)
    u = A.GpuUniform(gpu, size)
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 7)]:
        data, offsets, lens = u.encode_chunks(syms.astype(dtype), L, kind, seed)
        od, oo, ol = orc.codec_encode_chunks(orc.CODEC_UNIFORM, syms, L, param=size, kind=kind, seed=seed)
        assert np.array_equal(lens, ol) and data.tobytes() == od.tobytes()
        back = u.decode_chunks(data, offsets, lens, n, L, dtype, kind, seed)
        assert np.array_equal(back, syms.astype(dtype))


@pytest.mark.parametrize("excl_max_bits,max_bits", [(0, 0), (1, 1), (6, 6), (20, 17), (47, 47), (64, 40)])
@pytest.mark.parametrize("dtype,L", [(np.uint64, 4096), (np.uint64, 32), (np.uint8, 128)])
def test_loguniform_fast_bit_exact(gpu, excl_max_bits, max_bits, dtype, L):
    rng = np.random.default_rng(excl_max_bits * 31 + L)
    mb = min(max_bits, 8 * np.dtype(dtype).itemsize)
    n = 23 * L + 3
    bits = rng.integers(0, mb + 1, size=n)
    x = rng.integers(0, 1 << 62, size=n, dtype=np.uint64) >> np.uint64(62 - mb) if mb else np.zeros(n, np.uint64)
    syms = np.where(bits == 0, np.uint64(0), x >> (np.uint64(mb) - bits.astype(np.uint64))).astype(np.uint64)
    lu = A.GpuLogUniform(gpu, excl_max_bits)
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 2)]:
        data, offsets, lens = lu.encode_chunks(syms.astype(dtype), L, kind, seed)
        od, oo, ol = orc.codec_encode_chunks(orc.CODEC_LOGUNIFORM, syms, L, param=excl_max_bits, kind=kind, seed=seed)
        assert np.array_equal(lens, ol) and data.tobytes() == od.tobytes()
        back = lu.decode_chunks(data, offsets, lens, n, L, dtype, kind, seed)
        assert np.array_equal(back, syms.astype(dtype))


def test_loguniform_fast_ones_and_zeros(gpu):
    """Runs of x = 1 (bits = 1: the Uniform(1) push whose bound is 2^56, the one LogUniform push that
    can take a byte back) and x = 0 between large values, every chunk against the oracle."""
    rng = np.random.default_rng(77)
    L, nch = 64, 400
    syms = rng.choice(np.array([0, 1, 1, 1, 2, 3, (1 << 46) + 5, (1 << 30) + 1], np.uint64), size=L * nch)
    lu = A.GpuLogUniform(gpu, 47)
    data, offsets, lens = lu.encode_chunks(syms, L)
    od, oo, ol = orc.codec_encode_chunks(orc.CODEC_LOGUNIFORM, syms, L, param=47)
    assert np.array_equal(lens, ol) and data.tobytes() == od.tobytes()
    assert np.array_equal(lu.decode_chunks(data, offsets, lens, len(syms), L), syms)


def test_uniform_loguniform_fast_errors_and_device_api(gpu):
    torch = pytest.importorskip("torch")
    with pytest.raises(A.AnsError) as e:  # x >= size on a fast chunk
        A.GpuUniform(gpu, 10).encode_chunks(np.array([3] * 300 + [10] + [2] * 211, np.uint64), 16)
    assert e.value.code == A.ANS_E_SYMBOL
    with pytest.raises(A.AnsError) as e:  # bits = 7 > excl_max_bits = 6
        A.GpuLogUniform(gpu, 6).encode_chunks(np.array([1] * 100 + [127] + [0] * 27, np.uint64), 32)
    assert e.value.code == A.ANS_E_SYMBOL
    with pytest.raises(A.AnsError) as e:  # 2^47: Uniform::new(2^47) > MAX_SIZE (src/codec.rs:35)
        A.GpuLogUniform(gpu, 64).encode_chunks(np.array([1] * 63 + [1 << 47], np.uint64), 32)
    assert e.value.code == A.ANS_E_NORM_RANGE
    # device-resident: slots equal the host container's streams, decode lossless
    rng = np.random.default_rng(3)
    stream = torch.cuda.Stream()
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    L, nch = 512, 200
    for codec, syms in [(A.GpuUniform(gpu, (1 << 40) + 7), rng.integers(0, (1 << 40) + 7, size=L * nch, dtype=np.uint64)),
                        (A.GpuLogUniform(gpu, 47), rng.integers(0, 1 << 46, size=L * nch, dtype=np.uint64) >>
                         rng.integers(0, 46, size=L * nch).astype(np.uint64))]:
        data, offsets, lens = codec.encode_chunks(syms, L)
        d_syms = torch.from_numpy(syms.view(np.int64)).cuda()
        cap = codec.slot_capacity(L)
        slots = torch.zeros(nch * cap, dtype=torch.uint8, device="cuda")
        d_lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
        codec.dev_encode(d_syms, 8, len(syms), L, slots, cap, d_lens, status, stream)
        out = torch.zeros_like(d_syms)
        codec.dev_decode(slots, None, cap, d_lens, len(syms), L, out, 8, status, stream)
        assert gpu.status(status, stream) == 0
        assert torch.equal(out, d_syms)
        ln = d_lens.cpu().numpy().astype(np.uint64)
        assert np.array_equal(ln, lens)
        h = slots.cpu().numpy().reshape(nch, cap)
        assert np.concatenate([h[c, :ln[c]] for c in range(nch)]).tobytes() == data.tobytes()
