"""GPU parity of the other static codecs of src/codec.rs (include/ans_capi.h section 4b):
IID<Uniform>, IID<LogUniform> (MaxBenfordIID's item), Independent<Categorical>, and
Categoricals beyond the table kernels (norm >= 2^32, nsym > 65536) — every chunk's bytes equal
to the oracle's (oracle/ans_oracle.c orc_codec_*), decode lossless and back at the initial
message, errors as the reference's asserts."""
import numpy as np
import pytest

import ans_amd as A
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    return A.Gpu(0)


def _check(enc, dec, oenc, odec, syms, chunk_len, dtype, kind, seed):
    s = np.asarray(syms).astype(dtype)
    data, offsets, lens = enc(s, chunk_len, kind, seed)
    od, oo, ol = oenc(np.asarray(syms, np.uint64), chunk_len, kind, seed)
    assert np.array_equal(lens, ol)
    assert data.tobytes() == od.tobytes()
    back = dec(data, offsets, lens, len(s), chunk_len, dtype, kind, seed)
    assert np.array_equal(back, s)
    assert np.array_equal(odec(od, oo, ol, len(s), chunk_len, kind, seed), np.asarray(syms, np.uint64))


@pytest.mark.parametrize("size", [1, 2, 3, 1000, (1 << 28) - 57, (1 << 40) + 7, 1 << 46])
@pytest.mark.parametrize("chunk_len", [1, 7, 4096])
def test_uniform_bit_exact(gpu, size, chunk_len):
    rng = np.random.default_rng(size % 1000 + chunk_len)
    syms = rng.integers(0, size, size=20000, dtype=np.uint64)
    u = A.GpuUniform(gpu, size)
    for dtype, kind, seed in [(np.uint64, A.GEN_ZEROS, 0), (np.uint64, A.GEN_RANDOM, 5)] + \
            ([(np.uint32, A.GEN_ZEROS, 0)] if size <= 1 << 32 else []):
        _check(lambda s, L, k, sd: u.encode_chunks(s, L, k, sd),
               lambda d, o, ln, n, L, dt, k, sd: u.decode_chunks(d, o, ln, n, L, dt, k, sd),
               lambda s, L, k, sd: orc.codec_encode_chunks(orc.CODEC_UNIFORM, s, L, param=size, kind=k, seed=sd),
               lambda d, o, ln, n, L, k, sd: orc.codec_decode_chunks(orc.CODEC_UNIFORM, d, o, ln, n, L, param=size,
                                                                     kind=k, seed=sd),
               syms, chunk_len, dtype, kind, seed)


def test_uniform_errors(gpu):
    with pytest.raises(A.AnsError) as e:
        A.GpuUniform(gpu, (1 << 46) + 1).encode_chunks(np.zeros(4, np.uint64), 2)
    assert e.value.code == A.ANS_E_NORM_RANGE  # Uniform::new asserts size <= MAX_SIZE (src/codec.rs:35)
    with pytest.raises(A.AnsError) as e:
        A.GpuUniform(gpu, 10).encode_chunks(np.array([3, 10, 2], np.uint64), 2)
    assert e.value.code == A.ANS_E_SYMBOL


def _benford(rng, n, max_bits):
    bits = rng.integers(0, max_bits + 1, size=n)
    x = rng.integers(0, 1 << 62, size=n, dtype=np.uint64) >> np.uint64(62 - max_bits)
    return np.where(bits == 0, np.uint64(0), x >> (np.uint64(max_bits) - bits.astype(np.uint64))).astype(np.uint64)


@pytest.mark.parametrize("excl_max_bits,max_bits", [(6, 6), (20, 17), (47, 47), (64, 40)])
@pytest.mark.parametrize("chunk_len", [1, 100, 4096])
def test_loguniform_bit_exact(gpu, excl_max_bits, max_bits, chunk_len):
    rng = np.random.default_rng(excl_max_bits * 100 + chunk_len)
    syms = _benford(rng, 15000, max_bits)
    lu = A.GpuLogUniform(gpu, excl_max_bits)
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 11)]:
        _check(lambda s, L, k, sd: lu.encode_chunks(s, L, k, sd),
               lambda d, o, ln, n, L, dt, k, sd: lu.decode_chunks(d, o, ln, n, L, dt, k, sd),
               lambda s, L, k, sd: orc.codec_encode_chunks(orc.CODEC_LOGUNIFORM, s, L, param=excl_max_bits, kind=k,
                                                           seed=sd),
               lambda d, o, ln, n, L, k, sd: orc.codec_decode_chunks(orc.CODEC_LOGUNIFORM, d, o, ln, n, L,
                                                                     param=excl_max_bits, kind=k, seed=sd),
               syms, chunk_len, np.uint64, kind, seed)


def test_loguniform_matches_host_codec_and_errors(gpu):
    """One chunk equals the host coder's IID<LogUniform> push (ans_amd.LogUniform over the
    two-phase scalar ABI) on the same initial message; the reference's asserts are errors."""
    rng = np.random.default_rng(1)
    syms = _benford(rng, 500, 30)
    m = A.Message.zeros()
    A.IID(A.LogUniform(31), len(syms)).push(m, [int(x) for x in syms])
    data, _, _ = A.GpuLogUniform(gpu, 31).encode_chunks(syms, len(syms))
    assert data.tobytes() == m.flatten()
    with pytest.raises(A.AnsError) as e:  # bits = 7 > excl_max_bits = 6
        A.GpuLogUniform(gpu, 6).encode_chunks(np.array([1, 127], np.uint64), 2)
    assert e.value.code == A.ANS_E_SYMBOL
    with pytest.raises(A.AnsError) as e:  # 2^47: Uniform::new(2^47) > MAX_SIZE
        A.GpuLogUniform(gpu, 64).encode_chunks(np.array([1 << 47], np.uint64), 1)
    assert e.value.code == A.ANS_E_NORM_RANGE


def _tables(rng):
    t = [rng.integers(1, 1 << 20, size=256).astype(np.uint64),
         rng.integers(0, 5, size=17).astype(np.uint64),
         rng.integers(1 << 30, 1 << 40, size=1000).astype(np.uint64),     # norm >= 2^32
         np.array([3, 1], np.uint64),
         rng.integers(1, 1 << 12, size=70000).astype(np.uint64)]          # nsym > 65536
    t[1][0] = 9
    return t


@pytest.mark.parametrize("chunk_len", [1, 33, 4096])
def test_independent_bit_exact(gpu, chunk_len):
    rng = np.random.default_rng(chunk_len)
    tables = _tables(rng)
    n = 30000
    tids = rng.integers(0, len(tables), size=n).astype(np.uint32)
    syms = np.zeros(n, np.uint64)
    for t, m in enumerate(tables):
        nz = np.flatnonzero(m)
        sel = tids == t
        p = m[nz].astype(np.float64)
        syms[sel] = rng.choice(nz, size=int(sel.sum()), p=p / p.sum())
    ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in tables])
    for kind, seed in [(A.GEN_ZEROS, 0), (A.GEN_RANDOM, 3)]:
        _check(lambda s, L, k, sd: ts.encode_chunks(tids, s, L, k, sd),
               lambda d, o, ln, n_, L, dt, k, sd: ts.decode_chunks(tids, d, o, ln, L, dt, k, sd),
               lambda s, L, k, sd: orc.codec_encode_chunks(orc.CODEC_INDEPENDENT, s, L, tables=tables, tids=tids,
                                                           kind=k, seed=sd),
               lambda d, o, ln, n_, L, k, sd: orc.codec_decode_chunks(orc.CODEC_INDEPENDENT, d, o, ln, n_, L,
                                                                      tables=tables, tids=tids, kind=k, seed=sd),
               syms, chunk_len, np.uint32, kind, seed)
    bad = syms.copy()
    bad[np.flatnonzero(tids == 1)[0]] = 17  # out of range for the 17-symbol table
    with pytest.raises(A.AnsError) as e:
        ts.encode_chunks(tids, bad.astype(np.uint32), chunk_len)
    assert e.value.code == A.ANS_E_SYMBOL


@pytest.mark.parametrize("which", ["norm_2^45", "nsym_100000"])
def test_wide_categorical_through_the_table_api(gpu, which):
    """Categoricals the u32 table kernels do not take run on the exact 64-bit kernels through
    the ordinary section-4 calls (host and device, fixed and variable chunks)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(7)
    masses = (rng.integers(1 << 30, 1 << 35, size=1000) if which == "norm_2^45"
              else rng.integers(1, 1 << 10, size=100000)).astype(np.uint64)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    assert gt.paths() == 0
    p = masses.astype(np.float64)
    syms = rng.choice(len(masses), size=50000, p=p / p.sum()).astype(np.uint32)
    data, offsets, lens = gt.encode_chunks(syms, 1000)
    od, oo, ol = orc.encode_chunks(masses, syms, 1000)
    assert np.array_equal(lens, ol) and data.tobytes() == od.tobytes()
    assert np.array_equal(gt.decode_chunks(data, offsets, lens, len(syms), 1000), syms)
    starts = np.array([0, 1, 5000, 5000, 20000, 50000], np.uint64)
    vd, vo, vl = gt.encode_var_chunks(syms, starts)
    for c in range(len(starts) - 1):
        a, b = int(starts[c]), int(starts[c + 1])
        # an empty chunk is the flattened initial message itself
        ref = orc.encode_chunks(masses, syms[a:b], b - a)[0].tobytes() if b > a else orc.Message.zeros().flatten()
        assert vd[int(vo[c]):int(vo[c]) + int(vl[c])].tobytes() == bytes(ref)
    assert np.array_equal(gt.decode_var_chunks(vd, vo, vl, starts), syms)
    # device-resident slot layout
    stream = torch.cuda.Stream()
    d_syms = torch.from_numpy(syms.view(np.int32)).cuda()
    cap = gt.slot_capacity(1000)
    slots = torch.zeros(50 * cap, dtype=torch.uint8, device="cuda")
    d_lens = torch.zeros(50, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    gt.dev_encode(d_syms, 4, len(syms), 1000, slots, cap, d_lens, status, stream)
    out = torch.zeros_like(d_syms)
    gt.dev_decode(slots, None, cap, d_lens, len(syms), 1000, out, 4, status, stream)
    assert gpu.status(status, stream) == 0
    assert torch.equal(out, d_syms)
    assert np.array_equal(d_lens.cpu().numpy().astype(np.uint64), ol)
