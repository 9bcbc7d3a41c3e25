#!/usr/bin/env python3
"""Benchmark: device-resident rANS encode+decode on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path over one batch: encode every chunk of the
synthetic iid symbol array (one reference Message per chunk, IID<Categorical>::push,
src/codec.rs:415-420) and decode it back (IID::pop, src/codec.rs:422-424).

Default workload = SURVEY.md §8d config C3 (BASELINE.json configs[2]): 2^30 u8 symbols,
256-symbol table (norm 139,224,331), chunk_len 4096, generated on the device by the
counter-based splitmix64 generator (so every rank's shard is a slice of one global
array).  `--gpus N` runs one process per GPU: under torch.distributed.run (WORLD_SIZE set,
which must equal N) or, without a launcher, by starting torch.distributed.run as a child
process before this process touches a GPU.  Each rank codes its own 2^30-symbol shard
(weak scaling, no collective on the data path).

value = total uncompressed symbol GiB of all ranks / (max-over-ranks time per step).
roofline: algorithmic bytes of the dominant kernel (n*w symbols + compressed stream
bytes) / its average launch time from HIP events on its stream.
cpu_baseline: the oracle (oracle/ans_oracle.c) timed on a bounded sample of the same
workload (rank 0, N=1 only).

Sub-objects outside the headline's timed region:
  c4    BASELINE.json configs[3] per rank (2^29 u16 symbols, 65,536-symbol table): at N=8
        the aggregate is exactly C4's 8 GiB over 8 GPUs.  Its own barrier-bracketed wall
        clock and HIP events; the decoder's L2 request rate against tools/l2rand.hip's ceiling.
  dense the C3 wire format (ans_dev_encode_dense + decode in place).
  host  C3 from and to page-locked host memory through ans_gpu_encode_chunks /
        ans_gpu_decode_chunks (N=1), beside the measured link rate.
"""
import argparse
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "shuffle-coding_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
HBM_COPY_GBS = 6290.0  # measured float4 copy (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "ANS encode+decode GiB/s (device-resident) at 1/2/4/8 MI355X; % HBM roofline"
CONFIGS = {
    # name: (masses fn name, log2 n per rank, symbol bytes, seed)
    "c3": ("c3_masses", 30, 1, 1),
    "c3p2": ("c3_pow2_masses", 30, 1, 1),  # C3's table quantised to norm 2^24
    "c3s": ("c3_small_masses", 30, 1, 1),  # ... to norm 32,749 (< 2^16: count-built dataset tables)
    "c3b": ("c3_big_masses", 30, 1, 1),  # ... to norm 2^32 - 5 (> 2^31)
    "c4": ("c4_masses", 29, 2, 2),
    "c4s": ("c4_small_masses", 29, 2, 2),  # 4,096 of C4's masses quantised to norm 65,521 (< 2^16)
    "c4b": ("c4_big_masses", 29, 2, 2),  # C4's table quantised to norm 2^32 - 5 (> 2^31)
}


def parse(argv=None):
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
    p.add_argument("--no-c4", action="store_true", help="skip the C4 sub-object")
    p.add_argument("--c4-log2n", type=int, default=29, help="symbols per rank of the C4 sub-object")
    p.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe-inclusive) sub-object")
    p.add_argument("--strong", action="store_true",
                   help="strong scaling: the config's 2^log2n symbols in total, split over the ranks")
    p.add_argument("--test-fail-rank", type=int, default=None, help=argparse.SUPPRESS)  # tests/test_bench.py only
    return p.parse_args(argv)


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 with no launcher around us: N ranks under torch.distributed.run, started as
    a CHILD process (this process has not touched a GPU and never execs).  The ranks inherit
    stdout, so rank 0's JSON line is the only line printed; the exit code is the launcher's
    (non-zero when any rank failed)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def lib_hash(A):
    h = hashlib.sha256()
    with open(A.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pmc_record(A, kernel_key, config, log2n, chunk_len, pattern="*pmc*.json"):
    """The rocprofv3 PMC record of `kernel_key` on the same workload from a committed summary
    (profiles/*pmc*.json, written by tools/pmc_summary.py --json; or, with pattern "*kstats*.json",
    the kernel-trace --stats averages written by tools/kstats_json.py), preferring one taken on
    this exact library build, then the latest round; (record, source file, same build) or
    (None, None, False)."""
    best = None
    mine = lib_hash(A)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel_key)
        if k is None or (d.get("config"), d.get("log2n"), d.get("chunk_len")) != (config, log2n, chunk_len):
            continue
        rank = (d.get("lib_hash") == mine, path)
        if best is None or rank > best[0]:
            best = (rank, k, os.path.relpath(path, ROOT))
    return (None, None, False) if best is None else (best[1], best[2], best[0][0])


def l2_ceiling():
    """The chip's random-gather ceiling (lane requests/s, 16-B loads from a 1-MiB table: C4's
    bucket table) from the latest committed tools/l2rand.hip run (profiles/*l2rand*.json)."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*l2rand*.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    return d.get("ceiling_lane_requests_per_s"), os.path.relpath(paths[-1], ROOT)


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


class Ctx:
    """Per-process state shared by the passes."""

    def __init__(self, A, torch, dist, rank, world, local, backend):
        self.A, self.torch, self.dist = A, torch, dist
        self.rank, self.world, self.local, self.backend = rank, world, local, backend
        self.gpu = A.Gpu(local)
        # all work on one explicit stream (torch's default stream handle is NULL, which the C ABI
        # reads as "the context's own stream"); HIP events are recorded on this same stream
        self.stream = torch.cuda.Stream()
        torch.cuda.set_stream(self.stream)
        self.status = torch.zeros(1, dtype=torch.int32, device="cuda")

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def agree(self, err, what):
        """Every rank reaches this collective once per phase, whether its phase succeeded or not
        (err: this rank's exception or None); if any rank failed, every rank leaves together
        with an error instead of the healthy ranks waiting in the next barrier for one that has
        gone (torchrun would only reap them at its own timeout)."""
        flags = self.gather([0.0 if err is None else 1.0])
        bad = [r for r, f in enumerate(flags) if f[0] > 0]
        if bad:
            mine = f": {type(err).__name__}: {err}" if err is not None else ""
            if self.world > 1:
                self.dist.destroy_process_group()
            raise SystemExit(f"rank {self.rank}: {what} failed on rank(s) {bad}{mine}")

    def gather(self, values):
        """Every rank's float values, as a list of lists (rank order)."""
        t = self.torch.tensor(values, dtype=self.torch.float64,
                              device="cuda" if self.backend == "nccl" else "cpu")
        if self.world == 1:
            return [values]
        parts = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [[float(v) for v in p.tolist()] for p in parts]


def workload(ctx, masses, sym_bytes, seed, start, n, L):
    torch, A = ctx.torch, ctx.A
    gt = A.GpuTable(ctx.gpu, A.Categorical(masses))
    cap = gt.slot_capacity(L)
    nchunks = -(-n // L)
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[sym_bytes]
    syms = torch.empty(n, dtype=dt, device="cuda")
    gt.dev_gen_iid(seed, start, n, syms, sym_bytes, ctx.stream)  # this rank's slice of the global array
    slots = torch.empty(nchunks * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    out = torch.empty_like(syms)
    return gt, cap, nchunks, syms, slots, lens, out


def timed_round_trips(ctx, gt, syms, sym_bytes, n, L, slots, cap, lens, out, steps, warmup, pre=None, fail_rank=None):
    """warmup untimed steps, then `steps` steps bracketed by barrier + synchronize on both
    sides; (wall seconds, mean encode ms, mean decode ms, pre()'s result) with HIP events on
    ctx.stream.  pre: work queued just before the warm-up (the dense pass), inside the same
    failure agreement.  fail_rank (--test-fail-rank, tests only): that rank's warm-up raises."""
    torch, stream, status = ctx.torch, ctx.stream, ctx.status

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        gt.dev_encode(syms, sym_bytes, n, L, slots, cap, lens, status, stream)
        if ev is not None:
            ev[1].record(stream)
        gt.dev_decode(slots, None, cap, lens, n, L, out, sym_bytes, status, stream)
        if ev is not None:
            ev[2].record(stream)

    # a launch that raises on one rank must not leave the others in a barrier: every rank runs
    # both barriers of the timed region whatever happens, then all agree on the outcome
    err, pre_out = None, None
    try:
        if pre is not None:
            pre_out = pre()
        if fail_rank == ctx.rank:
            raise RuntimeError("--test-fail-rank")
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 (reported to every rank by ctx.agree)
        err = e
    ctx.agree(err, "warm-up")
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        for k in range(steps):
            step(events[k])
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        err = e
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    ctx.agree(err, "timed steps")
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))
    return elapsed, enc_ms, dec_ms, pre_out


def dense_pass(ctx, gt, syms, sym_bytes, n, L, nchunks, slots, cap, steps, warmup):
    """The dense container (the wire format) device-resident: ans_dev_encode_dense (encode into
    the slots, scan the lengths, pack) then ans_dev_decode_chunks reading the packed container in
    place; HIP events on the bench stream, outside the headline's timed region."""
    torch, stream, status = ctx.torch, ctx.stream, ctx.status
    offs = torch.empty(ctx.A.dense_offsets_entries(nchunks), dtype=torch.int64, device="cuda")
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

    def finish():  # (after the headline: no host synchronisation between the two passes)
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
    return finish


def kernel_name(A, gt, which, sym_bytes):
    if which == "decode":
        return "k_decode" + {"global": "_g", "wide": "_w"}.get(gt.decode_kernel(sym_bytes), "")
    return "k_encode" + ("_w" if gt.paths() & A.ANS_PATH_ENC_WIDE else "")


def c4_pass(ctx, args):
    """BASELINE.json configs[3] on this rank: 2^c4_log2n u16 symbols at the global index
    rank * 2^c4_log2n (seed 2), the 65,536-symbol table, chunk 4096.  The same barrier-bracketed
    timing as the headline (its own region), the kernels' HIP-event means, and the round trip
    verified.  Returns this rank's raw numbers (combined over ranks by the caller)."""
    A, torch = ctx.A, ctx.torch
    _, _, sym_bytes, seed = CONFIGS["c4"]
    n = 1 << args.c4_log2n
    L = args.chunk_len
    masses = A.c4_masses()
    err = None
    try:
        gt, cap, nchunks, syms, slots, lens, out = workload(ctx, masses, sym_bytes, seed, ctx.rank * n, n, L)
    except Exception as e:  # noqa: BLE001
        err = e
    ctx.agree(err, "c4 setup")
    elapsed, enc_ms, dec_ms, _ = timed_round_trips(ctx, gt, syms, sym_bytes, n, L, slots, cap, lens, out,
                                                   args.steps, min(args.warmup, 5))
    comp = 0.0
    try:
        st = ctx.gpu.status(ctx.status, ctx.stream)
        bad = 1.0 if (st != 0 or not torch.equal(out, syms)) else 0.0
        comp = float(lens.to(torch.int64).sum().item())
    except Exception:  # noqa: BLE001 (reported in the caller's gather)
        bad = 1.0
    names =(kernel_name(A, gt, "encode", sym_bytes), kernel_name(A, gt, "decode", sym_bytes))
    del syms, slots, lens, out
    torch.cuda.empty_cache()
    return [elapsed, enc_ms, dec_ms, comp, bad], names, n, masses


def c4_l2_share(masses):
    """The share of k_decode_w's bucket lookups that go to L2.  Its compact buckets have the finest
    width 2^cs with at most 2^17 of them (ans_kernels.hip build_fast_table); kWideDecBktLds =
    (160 KiB - 67,584 B of ring) / 16 = 6,016 buckets fit in LDS (ans_wide.hpp), staged at width
    2^(cs+1) when the table has more buckets and at most 1/256 of the staged cf lies past a staged
    bucket's five candidates (such lookups re-fetch their global bucket); cf is uniform."""
    m = np.asarray(masses, dtype=np.int64)
    cum = np.concatenate([[0], np.cumsum(m), np.full(5, m.sum())])
    norm = int(cum[len(m)])
    nlds = (160 * 1024 - 67584) // 16
    cs = 0
    while ((norm - 1) >> cs) + 1 > (1 << 17):
        cs += 1
    nb = ((norm - 1) >> cs) + 1
    if nb <= nlds:
        return 0.0
    ls = cs + 1
    nl = min(((norm - 1) >> ls) + 1, nlds)
    b0 = np.arange(nl, dtype=np.int64) << ls
    b1 = np.minimum(b0 + (1 << ls), norm)
    s0 = np.searchsorted(cum[:len(m) + 1], b0, side="right") - 1
    far = np.maximum(0, b1 - np.maximum(cum[s0 + 5], b0)).sum()
    covered = int((b1 - b0).sum())
    if far * 256 > covered:
        ls, covered, far = cs, min(nlds << cs, norm), 0
    return 1.0 - (covered - far) / norm


def c4_summary(rows, names, n, masses, args, world):
    """The c4 sub-object from every rank's [elapsed, enc_ms, dec_ms, comp, bad]."""
    sym_bytes = 2
    wall = max(r[0] for r in rows)
    share = c4_l2_share(masses)
    norm = int(np.asarray(masses, dtype=np.int64).sum())
    per = []
    for r in rows:
        alg = n * sym_bytes + r[3]
        per.append({"encode_ms": r[1], "decode_ms": r[2], "dec_frac": alg / (r[2] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    "enc_frac": alg / (r[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, "req_s": n * share / (r[2] * 1e-3)})
    ceil, ceil_src = l2_ceiling()
    r0 = per[0]
    out = {
        "workload": f"C4: 2^{args.c4_log2n} iid u16 symbols per GPU ({world * n * sym_bytes / 2**30:g} GiB "
                    f"over {world} GPU{'s' if world > 1 else ''}), 65536-symbol Categorical (norm {norm}), "
                    f"chunk_len {args.chunk_len}",
        "value": round(world * n * sym_bytes / (wall / args.steps) / 2**30, 3),
        "unit": "GiB/s",
        "ms_per_step": round(1e3 * wall / args.steps, 4),
        "per_gpu_gib_s": round(n * sym_bytes / (wall / args.steps) / 2**30, 3),
        "encode_ms": round(r0["encode_ms"], 4),
        "decode_ms": round(r0["decode_ms"], 4),
        "compressed_bytes_per_symbol": round(rows[0][3] / n, 5),
        "kernels": {"encode": names[0], "decode": names[1]},
        "roofline": {
            "bound": "l2-requests (decode: one random 16-B bucket gather per symbol on the chain, "
                     "past the buckets staged in LDS)",
            "decode_l2_share_of_lookups": round(share, 4),
            "decode_hbm_frac": round(r0["dec_frac"], 4),
            "encode_hbm_frac": round(r0["enc_frac"], 4),
            "decode_l2_req_per_s": round(r0["req_s"]),
            "l2_ceiling_req_per_s": ceil,
            "l2_req_frac": None if not ceil else round(r0["req_s"] / ceil, 4),
            "l2_ceiling_src": ceil_src,
        },
    }
    if world > 1:
        out["per_rank"] = {
            "ms_per_step": {"min": round(1e3 * min(r[0] for r in rows) / args.steps, 4),
                            "max": round(1e3 * wall / args.steps, 4)},
            "decode_hbm_frac": {"min": round(min(p["dec_frac"] for p in per), 4),
                                "max": round(max(p["dec_frac"] for p in per), 4)},
            "l2_req_frac": None if not ceil else {"min": round(min(p["req_s"] for p in per) / ceil, 4),
                                                  "max": round(max(p["req_s"] for p in per) / ceil, 4)},
        }
    return out


def link_rate(torch, nbytes):
    """Page-locked <-> device copy rates (GB/s): each direction alone, then both at once on two
    streams (a host round trip moves every byte once each way)."""
    h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, reps=3):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best

    def both():
        with torch.cuda.stream(s1):
            d_a.copy_(h_src, non_blocking=True)
        with torch.cuda.stream(s2):
            h_dst.copy_(d_b, non_blocking=True)

    h2d = timed(lambda: d_a.copy_(h_src, non_blocking=True))
    d2h = timed(lambda: h_dst.copy_(d_b, non_blocking=True))
    bi = timed(both)
    return {"h2d_gb_s": round(nbytes / h2d / 1e9, 2), "d2h_gb_s": round(nbytes / d2h / 1e9, 2),
            "both_ways_gb_s_each": round(nbytes / bi / 1e9, 2), "bytes": nbytes}


def host_pass(ctx, gt, d_syms, n, L, reps=3):
    """C3 from and to page-locked host memory through the C ABI's host-buffer entries
    (ans_gpu_encode_chunks -> dense container in host memory -> ans_gpu_decode_chunks), the
    north_star's "starts and ends in host memory" path; best of `reps` per direction."""
    import ctypes
    A, torch = ctx.A, ctx.torch
    lib = A.lib()
    nch = -(-n // L)
    cap = gt.slot_capacity(L) * nch
    hs = A.pinned_empty(n, np.uint8)
    torch.from_numpy(hs).copy_(d_syms.view(torch.uint8).cpu())
    ho = A.pinned_empty(cap, np.uint8)
    hb = A.pinned_empty(n, np.uint8)
    offs = np.zeros(nch, np.uint64)
    lens = np.zeros(nch, np.uint64)
    total = ctypes.c_uint64(0)
    te, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        A._check(lib.ans_gpu_encode_chunks(gt.h, hs.ctypes.data, 1, n, L, ho.ctypes.data, cap, offs.ctypes.data,
                                           lens.ctypes.data, ctypes.byref(total)), "ans_gpu_encode_chunks")
        t1 = time.perf_counter()
        A._check(lib.ans_gpu_decode_chunks(gt.h, ho.ctypes.data, total.value, offs.ctypes.data, lens.ctypes.data,
                                           n, L, A.GEN_ZEROS, hb.ctypes.data, 1), "ans_gpu_decode_chunks")
        t2 = time.perf_counter()
        te.append(t1 - t0)
        td.append(t2 - t1)
    ok = bool(np.array_equal(hb, hs))
    e, d = min(te), min(td)
    out = {
        "what": "C3 through ans_gpu_encode_chunks / ans_gpu_decode_chunks on page-locked host buffers "
                "(symbols in host memory -> dense container in host memory -> symbols in host memory); "
                f"best of {reps}",
        "encode_gib_s": round(n / e / 2**30, 3),
        "decode_gib_s": round(n / d / 2**30, 3),
        "gib_s": round(n / (e + d) / 2**30, 3),
        "encode_ms": [round(1e3 * x, 2) for x in te],
        "decode_ms": [round(1e3 * x, 2) for x in td],
        "container_bytes": int(total.value),
        "link": link_rate(torch, 1 << 30),
        "ok": ok,
    }
    del hs, ho, hb
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU, the two must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on device 0, and
    # gloo instead of RCCL for the barrier / gather (the data path has no collective)
    if os.environ.get("BENCH_SHARE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("BENCH_BACKEND", "nccl")

    import torch
    import torch.distributed as dist
    import ans_amd as A

    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    ctx = Ctx(A, torch, dist, rank, world, local, backend)

    masses_name, log2n, sym_bytes, seed = CONFIGS[args.config]
    if args.log2n is not None:
        log2n = args.log2n
    if args.strong:  # the 2^log2n-symbol array split into whole-chunk ranges, one per rank
        import shards
        total_n = 1 << log2n
        start, end, _, _ = shards.shard_symbols(total_n, args.chunk_len, world, rank)
        n = end - start
    else:
        n = 1 << log2n
        start, total_n = rank * n, world * n
    L = args.chunk_len
    masses = getattr(A, masses_name)()
    err = None
    try:
        gt, cap, nchunks, syms, slots, lens, out = workload(ctx, masses, sym_bytes, seed, start, n, L)
    except Exception as e:  # noqa: BLE001
        err = e
    ctx.agree(err, "setup")

    # The dense-container pass (the wire format: its own events, read and verified after the
    # headline) is queued just before the headline, with no host synchronisation in between.
    # The GPU's clocks fall back after even a short idle gap and take ~50 ms of continuous work
    # to recover: with the dense pass read out in between, the driver's --warmup 5 left the
    # headline 2.5% below its steady state (497 vs 511 GiB/s at --warmup 30 on one box; queued
    # this way, 513 at either).
    # (20 warm-up steps of its own at least: ~50 ms, the clocks' settling time)
    pre = None if args.no_dense else (lambda: dense_pass(ctx, gt, syms, sym_bytes, n, L, nchunks, slots, cap,
                                                         min(args.steps, 10), max(args.warmup, 20)))
    elapsed, enc_ms, dec_ms, dense_finish = timed_round_trips(ctx, gt, syms, sym_bytes, n, L, slots, cap, lens,
                                                              out, args.steps, args.warmup, pre=pre,
                                                              fail_rank=args.test_fail_rank)
    dense = None if dense_finish is None else dense_finish()
    dense_bad = dense is not None and not dense.pop("ok")

    # ---- verification (outside the timed region); every rank learns whether any failed (a rank
    # whose check itself raises reports a failure in the same gather instead of leaving it)
    st, comp_bytes = 0, 0
    try:
        st = ctx.gpu.status(ctx.status, ctx.stream)
        bad = 1.0 if (dense_bad or st != 0 or not torch.equal(out, syms)) else 0.0
        comp_bytes = int(lens.to(torch.int64).sum().item())
    except Exception:  # noqa: BLE001
        bad = 1.0
    del slots, out
    torch.cuda.empty_cache()

    c4, c4_row = None, None
    if args.config != "c4" and not args.no_c4:
        c4_row, c4_names, c4_n, c4_masses = c4_pass(ctx, args)  # [elapsed, enc_ms, dec_ms, comp, bad]

    # every rank's [elapsed, bad, enc_ms, dec_ms, n, comp_bytes] (+ its c4 row)
    rows = ctx.gather([elapsed, bad, enc_ms, dec_ms, float(n), float(comp_bytes)] + (c4_row or []))
    if any(r[1] > 0 for r in rows) or (c4_row is not None and any(r[10] > 0 for r in rows)):
        msg = A.lib().ans_status_string(st).decode() if st else "decoded symbols differ (this or another rank)"
        raise SystemExit(f"rank {rank}: round trip failed ({msg})")
    if c4_row is not None:
        c4 = c4_summary([r[6:] for r in rows], c4_names, c4_n, c4_masses, args, world)

    host = None
    if world == 1 and not args.no_host and args.config in ("c3", "c3p2", "c3s", "c3b"):
        host = host_pass(ctx, gt, syms, n, L)
        if not host.pop("ok"):
            raise SystemExit("host-memory round trip failed")

    wall = max(r[0] for r in rows)
    ms_per_step = 1e3 * wall / args.steps
    total_sym_bytes = total_n * sym_bytes
    value = total_sym_bytes / (wall / args.steps) / 2**30

    dom_name, dom_ms = ("decode", dec_ms) if dec_ms >= enc_ms else ("encode", enc_ms)
    dom_kernel = kernel_name(A, gt, dom_name, sym_bytes)
    other_name = "encode" if dom_name == "decode" else "decode"
    other_kernel = kernel_name(A, gt, other_name, sym_bytes)
    alg_bytes = n * sym_bytes + comp_bytes  # per launch, encode and decode alike
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    # the PMC records are per-rank workloads of 2^log2n symbols (not a strong-scaling share)
    strong_split = args.strong and world > 1

    def valu_of(kernel, ms):
        rec, src, same = (None, None, False) if strong_split else pmc_record(A, kernel, args.config, log2n, L)
        if rec is None or "valu_per_wave" not in rec.get("derived", {}):
            return rec, src, None
        # one wave = 64 lanes = 64 chunks, one VALU wave-instruction per lane-step;
        # issue capacity: 4 SIMDs per CU, one wave64 VALU instruction per 4 cycles each (the
        # 4-cycle class of tools/microbench.hip; simple 32-bit adds/logic issue in 2)
        d = rec["derived"]
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        wave_instr = d["valu_per_wave"] * nchunks / 64
        clk = d.get("clock_ghz")
        return rec, src, {
            "kernel": kernel,
            "pmc_same_build": same,  # False: the counts are another build's (the latest committed record)
            "instr_per_symbol": round(d["valu_per_wave"] / L, 2),
            "frac_at_2.4GHz": round(wave_instr * 4 / (cus * 4 * 2.4e9 * ms * 1e-3), 4),
            "clock_ghz_pmc": None if clk is None else round(clk, 3),
            "frac_at_pmc_clock": None if clk is None else round(wave_instr * 4 / (cus * 4 * clk * 1e9 * d["duration_ns"] * 1e-9), 4),
        }

    rec, rec_src, valu = valu_of(dom_kernel, dom_ms)
    _, _, valu_other = valu_of(other_kernel, enc_ms if other_name == "encode" else dec_ms)
    traffic = None if rec is None else rec.get("hbm_bytes_per_launch")
    pmc_same = bool(valu and valu["pmc_same_build"])
    # the same fraction from the committed rocprofv3 --kernel-trace --stats average of the
    # dominant kernel (profiles/*kstats*.json), beside the HIP-event one
    ks, ks_src, ks_same = (None, None, False) if strong_split else pmc_record(A, dom_kernel, args.config, log2n, L,
                                                                               pattern="*kstats*.json")
    ks_ns = None if ks is None else ks.get("avg_ns")
    hbm_frac = achieved / HBM_PEAK_GBS
    # what binds: the VALU issue fraction (PMC instruction count at 4 cycles per wave64
    # instruction) when it exceeds the HBM fraction, as it does for the integer coding kernels;
    # only from PMC counts of this very build (another build's counts name no bound)
    if valu and valu["pmc_same_build"]:
        bound = "valu-issue" if valu["frac_at_2.4GHz"] > hbm_frac else "hbm"
    else:
        bound = "unknown (no PMC record of this build)"

    if rank == 0:
        per_frac = [(r[4] * sym_bytes + r[5]) / (max(r[2], r[3]) * 1e-3) / 1e9 / HBM_PEAK_GBS for r in rows]
        line = {
            "metric": METRIC,
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
                "symbols_per_rank": [int(r[4]) for r in rows],
                "symbols_total": total_n,
                "symbol_bytes": sym_bytes,
                "chunk_len": L,
                "chunks_per_gpu": nchunks,
                "parallelism": f"chunk-sharded x{world}, no collective",
            },
            "per_rank_ms_per_step": {"min": round(1e3 * min(r[0] for r in rows) / args.steps, 4),
                                     "max": round(ms_per_step, 4)},
            "encode_ms": round(enc_ms, 4),
            "decode_ms": round(dec_ms, 4),
            "encode_gib_s": round(n * sym_bytes / (enc_ms * 1e-3) / 2**30, 3),
            "decode_gib_s": round(n * sym_bytes / (dec_ms * 1e-3) / 2**30, 3),
            "compressed_bytes_per_symbol": round(comp_bytes / n, 5),
            "dense": dense,
            "c4": c4,
            "host": host,
            "parity": "round trip verified on device; byte parity vs the oracle: tests/test_gpu_parity.py",
            "roofline": {
                "bound": bound,
                "kernel": dom_kernel,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(hbm_frac, 4),
                "frac_rocprof": None if not ks_ns else round(alg_bytes / ks_ns / HBM_PEAK_GBS, 4),
                "rocprof_avg_ns": ks_ns,
                "rocprof_src": ks_src,
                "rocprof_same_build": ks_same,
                "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),  # vs 6.29 TB/s float4 copy
                "traffic": None if traffic is None else round(traffic),
                "traffic_over_alg": None if traffic is None else round(traffic / alg_bytes, 3),
                "traffic_src": rec_src,
                "pmc_same_build": pmc_same,
                # 0.70 of 8 TB/s at this workload's bytes per symbol, against the chip's VALU issue
                # rate (256 CU x 4 SIMD x 16 lanes x 2.4 GHz): the most VALU per symbol, encode and
                # decode each, that the north_star target allows
                "valu_per_symbol_budget_at_0.70": round(
                    256 * 4 * 16 * 2.4e9 / (0.70 * HBM_PEAK_GBS * 1e9 / (alg_bytes / n)), 1),
                "valu": valu,
                "valu_other": valu_other,
                "per_rank_frac": {"min": round(min(per_frac), 4), "max": round(max(per_frac), 4)},
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(masses, sym_bytes, seed, L, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
