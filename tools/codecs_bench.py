"""Rates of the codecs beside Categorical on the GPU: Independent<Categorical>
with a table per position (src/codec.rs:366-403), IID<Uniform> (src/codec.rs:13-49) and
IID<LogUniform(47)> (src/codec.rs:561-611, MaxBenfordIID's item).

Device-resident (include/ans_capi.h 4b ans_dev_*): symbols and table ids already in HBM, streams
into slots, HIP events on the call's stream around each kernel pass, mean of `reps` passes after
`warm` untimed ones; every pass's round trip is verified once at the end.  Set ANS_CODECS_EXACT=1
to time the exact 64-bit kernels instead (the same bytes).  The host-buffer calls (upload,
allocation and download included) are timed once per workload beside them.  Prints one JSON line.
usage: python tools/codecs_bench.py [log2n_independent=28] [log2n_uniform=26]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402


def timed_device(enc, dec, check, reps=10, warm=3):
    stream = torch.cuda.current_stream()
    for _ in range(warm):
        enc()
        dec()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    for e in ev:
        e[0].record(stream)
        enc()
        e[1].record(stream)
        dec()
        e[2].record(stream)
    torch.cuda.synchronize()
    te = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    td = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    check()
    return te, td


def line(n, sym_bytes, te, td, comp, **kw):
    return dict(symbols=n, sym_bytes=sym_bytes, encode_ms=round(te, 4), decode_ms=round(td, 4),
                gib_s=round(n * sym_bytes / ((te + td) * 1e-3) / 2**30, 3),
                encode_gib_s=round(n * sym_bytes / (te * 1e-3) / 2**30, 3),
                decode_gib_s=round(n * sym_bytes / (td * 1e-3) / 2**30, 3),
                compressed_bytes_per_symbol=round(comp / n, 5), **kw)


def device_case(gpu, codec, syms_np, L, w, tids_np=None, stream=None):
    """syms_np / tids_np: host arrays, or device tensors already in HBM (generated there)"""
    stream = stream or torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    n = len(syms_np)
    nch = n // L
    if isinstance(syms_np, torch.Tensor):
        d_syms, d_tids = syms_np, tids_np
    else:
        d_syms = torch.from_numpy(syms_np.view({1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[w])).cuda()
        d_tids = None if tids_np is None else torch.from_numpy(tids_np.astype(np.uint8)).cuda()
    cap = codec.slot_capacity(L)
    slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty_like(d_syms)
    if d_tids is None:
        enc = lambda: codec.dev_encode(d_syms, w, n, L, slots, cap, lens, status, stream)  # noqa: E731
        dec = lambda: codec.dev_decode(slots, None, cap, lens, n, L, out, w, status, stream)  # noqa: E731
    else:
        enc = lambda: codec.dev_encode(d_tids, d_syms, w, n, L, slots, cap, lens, status, stream)  # noqa: E731
        dec = lambda: codec.dev_decode(d_tids, slots, None, cap, lens, n, L, out, w, status, stream)  # noqa: E731

    def check():
        assert gpu.status(status, stream) == 0
        assert torch.equal(out, d_syms), "round trip"

    te, td = timed_device(enc, dec, check)
    comp = int(lens.to(torch.int64).sum().item())
    del slots, out, d_syms
    torch.cuda.set_stream(torch.cuda.default_stream())
    torch.cuda.empty_cache()
    return te, td, comp


def host_case(enc, dec, n, w):
    t0 = time.perf_counter()
    e = enc()
    t1 = time.perf_counter()
    dec(e)
    t2 = time.perf_counter()
    return {"host_api_gib_s": round(n * w / (t2 - t0) / 2**30, 3)}


def main():
    li = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    lu = int(sys.argv[2]) if len(sys.argv) > 2 else 26
    L = 4096
    rng = np.random.default_rng(3)
    g = A.Gpu(0)
    res = {"chunk_len": L, "kernels": "exact" if os.environ.get("ANS_CODECS_EXACT") == "1" else "fast",
           "what": "device-resident ans_dev_* encode + decode, HIP-event means of 10 passes; GiB/s of symbol bytes"}

    # Independent: five 256-symbol tables (norm in the fast range), position k uses table k % 5;
    # the symbols of table t drawn on the device (its counter-based iid generator, seed t) and
    # kept at the positions k = t mod 5
    n = 1 << li
    ms = [rng.integers(1, 1 << 16, 256).astype(np.uint64) for _ in range(5)]
    ts = A.GpuTableSet(g, [A.Categorical(m) for m in ms])
    stream = torch.cuda.Stream()
    d_tids = (torch.arange(n, device="cuda", dtype=torch.int64) % 5).to(torch.uint8)
    d_syms = torch.empty(n, dtype=torch.uint8, device="cuda")
    tmp = torch.empty(n, dtype=torch.uint8, device="cuda")
    for t in range(5):
        A.GpuTable(g, A.Categorical(ms[t])).dev_gen_iid(t, 0, n, tmp, 1, stream)
        torch.cuda.synchronize()
        d_syms[t::5] = tmp[t::5]
    del tmp
    torch.cuda.synchronize()
    te, td, comp = device_case(g, ts, d_syms, L, 1, d_tids, stream)
    res["independent"] = line(n, 1, te, td, comp, tables=5, table_symbols=256, tableset_fast=ts.fast())
    if os.environ.get("CODECS_LANES_AB") == "1":  # both workgroup layouts, same box (ans_gpu_tableset_lanes)
        for lanes in (256, 1024):
            ts.lanes(lanes)
            te, td, comp = device_case(g, ts, d_syms, L, 1, d_tids, stream)
            res[f"independent_lanes{lanes}"] = line(n, 1, te, td, comp)
        ts.lanes(0)
    if li <= 26:
        tids, syms = d_tids.cpu().numpy().astype(np.uint32), d_syms.cpu().numpy()
        res["independent"].update(host_case(lambda: ts.encode_chunks(tids, syms, L),
                                            lambda e: ts.decode_chunks(tids, *e, L, np.uint8), n, 1))
    del d_tids, d_syms
    torch.cuda.empty_cache()

    # Uniform(2^40) (a power of two: shifts) and Uniform(2^40 + 7) (the magic-reciprocal division)
    n = 1 << lu
    for size, key in [(1 << 40, "uniform_2^40"), ((1 << 40) + 7, "uniform_2^40+7")]:
        gu = A.GpuUniform(g, size)
        xs = rng.integers(0, size, n, dtype=np.uint64)
        te, td, comp = device_case(g, gu, xs, L, 8)
        res[key] = line(n, 8, te, td, comp)

    # LogUniform(47): bit lengths uniform over 0..47, the bits below the top one uniform
    bits = rng.integers(0, 48, n)
    low = rng.integers(0, 1 << 46, n, dtype=np.uint64)
    sh = np.maximum(bits - 1, 0).astype(np.uint64)
    xs = np.where(bits == 0, 0, (np.uint64(1) << sh) | (low & ((np.uint64(1) << sh) - np.uint64(1)))).astype(np.uint64)
    gl = A.GpuLogUniform(g, 47)
    te, td, comp = device_case(g, gl, xs, L, 8)
    res["loguniform_47"] = line(n, 8, te, td, comp)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
