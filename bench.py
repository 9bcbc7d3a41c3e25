#!/usr/bin/env python3
"""Benchmark: device-resident rANS encode+decode on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path over one batch: encode every chunk of the
synthetic iid symbol array (one reference Message per chunk, IID<Categorical>::push,
src/codec.rs:415-420) and decode it back (IID::pop, src/codec.rs:422-424).

Default workload = SURVEY.md §8d config C3 (BASELINE.json configs[2]): 2^30 u8 symbols,
256-symbol table (norm 139,224,331), chunk_len 4096, generated on the device by the
counter-based splitmix64 generator (so every rank's shard is a slice of one global
array).  With --gpus N (torchrun, one process per GPU) each rank codes its own 2^30
symbol shard (weak scaling, no collective on the data path).

value = total uncompressed symbol GiB of all ranks / (max-over-ranks time per step).
roofline: algorithmic bytes of the dominant kernel (n*w symbols + compressed stream
bytes) / its average launch time from HIP events on its stream.
cpu_baseline: the oracle (oracle/ans_oracle.c, single thread) timed on a bounded
sample of the same workload (rank 0, N=1 only).
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "shuffle-coding_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ans_amd as A  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
CONFIGS = {
    # name: (masses fn, log2 n per rank, symbol bytes, seed)
    "c3": (A.c3_masses, 30, 1, 1),
    "c3p2": (A.c3_pow2_masses, 30, 1, 1),  # C3's table quantised to norm 2^24
    "c4": (A.c4_masses, 29, 2, 2),
}
HBM_COPY_GBS = 6290.0  # measured float4 copy (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)  # the clocks ramp over the first ~5 steps
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--log2n", type=int, default=None, help="symbols per rank = 2^log2n (default: the config's)")
    p.add_argument("--chunk-len", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-dense", action="store_true", help="skip the dense-container pass")
    p.add_argument("--strong", action="store_true",
                   help="strong scaling: the config's 2^log2n symbols in total, split over the ranks")
    return p.parse_args()


def lib_hash():
    h = hashlib.sha256()
    with open(A.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pmc_record(kernel_key, config, log2n, chunk_len):
    """The rocprofv3 PMC record of `kernel_key` on the same workload from a committed summary
    (profiles/*pmc*.json, written by tools/pmc_summary.py --json), preferring one taken on this
    exact library build, then the latest round; (record, source file) or (None, None)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel_key)
        if k is None or (d.get("config"), d.get("log2n"), d.get("chunk_len")) != (config, log2n, chunk_len):
            continue
        rank = (d.get("lib_hash") == lib_hash(), path)
        if best is None or rank > best[0]:
            best = (rank, k, os.path.relpath(path, ROOT))
    return (None, None) if best is None else (best[1], best[2])


def cpu_baseline(masses, sym_bytes, seed, chunk_len, target_s):
    """Oracle (single thread) encode+decode on the first chunks of the same workload."""
    from oracle import oracle as orc
    pilot = 64 * chunk_len
    syms = orc.gen_iid(masses, seed, 0, pilot)
    t0 = time.perf_counter()
    d, o, l = orc.encode_chunks(masses, syms, chunk_len)
    orc.decode_chunks(masses, d, o, l, pilot, chunk_len)
    per_sym = (time.perf_counter() - t0) / pilot
    nchunks = max(64, int(target_s / per_sym / chunk_len))
    n = nchunks * chunk_len
    syms = orc.gen_iid(masses, seed, 0, n)
    t0 = time.perf_counter()
    d, o, l = orc.encode_chunks(masses, syms, chunk_len)
    t1 = time.perf_counter()
    back = orc.decode_chunks(masses, d, o, l, n, chunk_len)
    t2 = time.perf_counter()
    assert np.array_equal(back, syms)
    out = {
        "value": n * sym_bytes / (t2 - t0) / 2**30,
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {nchunks} chunks x {chunk_len} symbols ({n} symbols) of the same workload; "
                  f"encode {t1 - t0:.2f}s + decode {t2 - t1:.2f}s, oracle/ans_oracle.c single thread",
    }
    # chunk-parallel on the host cores: one contiguous chunk range per thread
    # (the oracle's ctypes calls release the GIL); about 3 s of work per thread
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, min(16, os.cpu_count() or 1))  # a GPU box's CPU share is 16
    per_thread = max(16, int(3.0 / per_sym / chunk_len))
    m = per_thread * chunk_len
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(lambda i: orc.gen_iid(masses, seed, i * m, m), range(threads)))
        t0 = time.perf_counter()
        enc = list(ex.map(lambda x: orc.encode_chunks(masses, x, chunk_len), parts))
        t1 = time.perf_counter()
        dec = list(ex.map(lambda e: orc.decode_chunks(masses, e[0], e[1], e[2], m, chunk_len), enc))
        t2 = time.perf_counter()
    assert all(np.array_equal(a, b) for a, b in zip(dec, parts))
    out["parallel"] = {
        "value": threads * m * sym_bytes / (t2 - t0) / 2**30,
        "cores": threads,
        "sample": f"{threads} threads x {per_thread} chunks; encode {t1 - t0:.2f}s + decode {t2 - t1:.2f}s",
    }
    return out


def dense_pass(gt, syms, sym_bytes, n, L, nchunks, slots, cap, status, stream, steps, warmup):
    """The dense container (the wire format) device-resident: ans_dev_encode_dense (encode into
    the slots, scan the lengths, pack) then ans_dev_decode_chunks reading the packed container in
    place; HIP events on the bench stream, outside the headline's timed region."""
    offs = torch.empty(A.dense_offsets_entries(nchunks), dtype=torch.int64, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    dense = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(syms)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        gt.dev_encode_dense(syms, sym_bytes, n, L, slots, cap, lens, offs, dense, status, stream)
        if ev is not None:
            ev[1].record(stream)
        gt.dev_decode(dense, offs, cap, lens, n, L, out, sym_bytes, status, stream)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(warmup):
        step()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for k in range(steps):
        step(events[k])
    torch.cuda.synchronize()
    enc = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    dec = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))
    ok = torch.equal(out, syms) and int(offs[nchunks].item()) == int(lens.to(torch.int64).sum().item())
    return {"encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
            "gib_s": round(n * sym_bytes / ((enc + dec) * 1e-3) / 2**30, 3),
            "container_bytes": int(offs[nchunks].item()),
            "what": "ans_dev_encode_dense (encode + length scan + pack) and ans_dev_decode_chunks on the "
                    "packed container in place; round trip verified",
            "ok": ok}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on device 0, and
    # gloo instead of RCCL for the barrier / max-over-ranks (the data path has no collective)
    if os.environ.get("BENCH_SHARE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    masses_fn, log2n, sym_bytes, seed = CONFIGS[args.config]
    if args.log2n is not None:
        log2n = args.log2n
    if args.strong:  # the 2^log2n-symbol array split into whole-chunk ranges, one per rank
        sys.path.insert(0, os.path.join(ROOT, "shuffle-coding_amd"))
        import shards
        total_n = 1 << log2n
        start, end, _, _ = shards.shard_symbols(total_n, args.chunk_len, world, rank)
        n = end - start
    else:
        n = 1 << log2n
        start, total_n = rank * n, world * n
    L = args.chunk_len
    nchunks = -(-n // L)
    masses = masses_fn()

    gpu = A.Gpu(local)
    gt = A.GpuTable(gpu, A.Categorical(masses))
    cap = gt.slot_capacity(L)
    # all work on one explicit stream (torch's default stream handle is NULL, which the C ABI
    # reads as "the context's own stream"); HIP events are recorded on this same stream
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[sym_bytes]
    syms = torch.empty(n, dtype=dt, device="cuda")
    gt.dev_gen_iid(seed, start, n, syms, sym_bytes, stream)  # this rank's slice of the global array
    slots = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty_like(syms)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        gt.dev_encode(syms, sym_bytes, n, L, slots, cap, lens, status, stream)
        if ev is not None:
            ev[1].record(stream)
        gt.dev_decode(slots, None, cap, lens, n, L, out, sym_bytes, status, stream)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # ---- verification (outside the timed region); every rank learns whether any failed
    st = gpu.status(status, stream)
    bad = 1.0 if (st != 0 or not torch.equal(out, syms)) else 0.0
    comp_bytes = int(lens.to(torch.int64).sum().item())

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))
    # (its own warmup: clocks drop while the slot pass is verified; at most 10 timed steps)
    dense = None if args.no_dense else dense_pass(gt, syms, sym_bytes, n, L, nchunks, slots, cap, status, stream,
                                                  min(args.steps, 10), args.warmup)
    if dense is not None and (not dense.pop("ok") or gpu.status(status, stream) != 0):
        bad = 1.0
    t = torch.tensor([elapsed, bad], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    per_rank = [elapsed]
    if world > 1:
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        per_rank = [float(x[0].item()) for x in parts]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if t[1].item() > 0:
        msg = A.lib().ans_status_string(st).decode() if st else "decoded symbols differ"
        raise SystemExit(f"rank {rank}: round trip failed ({msg})")
    elapsed = float(t[0].item())
    ms_per_step = 1e3 * elapsed / args.steps
    total_sym_bytes = total_n * sym_bytes
    value = total_sym_bytes / (elapsed / args.steps) / 2**30

    alg_bytes = n * sym_bytes + comp_bytes  # per launch, encode and decode alike
    dom_name, dom_ms = ("decode", dec_ms) if dec_ms >= enc_ms else ("encode", enc_ms)
    suffix = {"global": "_g", "wide": "_w"}.get(gt.decode_kernel(sym_bytes), "") if dom_name == "decode" else \
        ("_w" if gt.paths() & A.ANS_PATH_ENC_WIDE else "")
    dom_kernel = f"k_{dom_name}{suffix}"
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    # the PMC records are per-rank workloads of 2^log2n symbols (not a strong-scaling share)
    rec, rec_src = (None, None) if (args.strong and world > 1) else pmc_record(dom_kernel, args.config, log2n, L)
    traffic = None if rec is None else rec.get("hbm_bytes_per_launch")
    valu = None
    if rec is not None and "valu_per_wave" in rec.get("derived", {}):
        # one wave = 64 lanes = 64 chunks, one VALU wave-instruction per lane-step;
        # issue capacity: 4 SIMDs per CU, one wave64 VALU instruction per 4 cycles each (the
        # 4-cycle class of tools/microbench.hip; simple 32-bit adds/logic issue in 2)
        d = rec["derived"]
        per_sym = d["valu_per_wave"] / L
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        wave_instr = d["valu_per_wave"] * nchunks / 64
        clk = d.get("clock_ghz")
        valu = {
            "instr_per_symbol": round(per_sym, 2),
            "frac_at_2.4GHz": round(wave_instr * 4 / (cus * 4 * 2.4e9 * dom_ms * 1e-3), 4),
            "clock_ghz_pmc": None if clk is None else round(clk, 3),
            "frac_at_pmc_clock": None if clk is None else round(wave_instr * 4 / (cus * 4 * clk * 1e9 * d["duration_ns"] * 1e-9), 4),
        }

    if rank == 0:
        line = {
            "metric": "ANS encode+decode GiB/s (device-resident) at 1/2/4/8 MI355X; % HBM roofline",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based splitmix64 iid symbols generated on device, SURVEY.md §8d)",
            "config": {
                "workload": f"{args.config.upper()}: 2^{log2n} iid u{8 * sym_bytes} symbols "
                            f"{'in total' if args.strong else 'per GPU'}, "
                            f"{len(masses)}-symbol Categorical (norm {int(masses.sum())}), chunk_len {L}",
                "symbols_per_gpu": n,
                "symbol_bytes": sym_bytes,
                "chunk_len": L,
                "chunks_per_gpu": nchunks,
                "parallelism": f"chunk-sharded x{world}, no collective",
            },
            "per_rank_ms_per_step": {"min": round(1e3 * min(per_rank) / args.steps, 4),
                                     "max": round(1e3 * max(per_rank) / args.steps, 4)},
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_gib_s": round(n * sym_bytes / (enc_ms * 1e-3) / 2**30, 3),
            "decode_gib_s": round(n * sym_bytes / (dec_ms * 1e-3) / 2**30, 3),
            "compressed_bytes_per_symbol": round(comp_bytes / n, 5),
            "dense": dense,
            "parity": "round trip verified on device; byte parity: tests/test_gpu_parity.py",
            "roofline": {
                "bound": "hbm",
                "kernel": dom_kernel,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),  # vs 6.29 TB/s float4 copy
                "traffic": None if traffic is None else round(traffic),
                "traffic_over_alg": None if traffic is None else round(traffic / alg_bytes, 3),
                "traffic_src": rec_src,
                "valu": valu,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(masses, sym_bytes, seed, L, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
