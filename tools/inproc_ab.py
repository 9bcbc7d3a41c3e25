"""Same-process A/B of two builds of the library on the C3 bench workload.

usage: python tools/inproc_ab.py <libdir A> <libdir B> [iters]
  AB_CONFIG=c4 AB_LOG2N=29: another bench config / size (default: C3 at its full size)
  AB_DENSE=1: the dense container (ans_dev_encode_dense, decode in place) instead of slots
  libdir: a directory under shuffle-coding_amd/ holding libshufflecoding_amd.so ("lib" = default)

Both builds are loaded side by side (RTLD_LOCAL, each registers its own code object) and run
alternately on the same device-resident symbols, so clocks and the box are shared; the kernel
times are HIP events on one explicit stream.  Prints the median encode / decode ms of each.
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "shuffle-coding_amd"))
import ans_amd as A  # noqa: E402
import bench  # noqa: E402


def load(d):
    L = ctypes.CDLL(os.path.join(HERE, "..", "shuffle-coding_amd", d, "libshufflecoding_amd.so"))
    for name, (res, args) in A.SIGNATURES.items():
        f = getattr(L, name, None)  # an older build may lack newer entry points
        if f is None:
            continue
        f.restype = res
        f.argtypes = args
    return L


def indep(dirs, iters, sync):
    """AB_CONFIG=indep: tools/codecs_bench.py's Independent workload (five 256-symbol tables,
    position k uses table k mod 5, 2^AB_LOG2N u8 symbols, default 30) on both builds."""
    n, L = 1 << int(os.environ.get("AB_LOG2N", 30)), 4096
    rng = np.random.default_rng(3)
    ms = [rng.integers(1, 1 << 16, 256).astype(np.uint64) for _ in range(5)]
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    libs = [load(d) for d in dirs]
    d_tids = (torch.arange(n, device="cuda", dtype=torch.int64) % 5).to(torch.uint8)
    syms = torch.empty(n, dtype=torch.uint8, device="cuda")
    setups = []
    for i, Lb in enumerate(libs):
        A._lib = Lb
        gpu = A.Gpu(0)
        if i == 0:
            tmp = torch.empty(n, dtype=torch.uint8, device="cuda")
            for t in range(5):
                A.GpuTable(gpu, A.Categorical(ms[t])).dev_gen_iid(t, 0, n, tmp, 1, stream)
                torch.cuda.synchronize()
                syms[t::5] = tmp[t::5]
            del tmp
        ts = A.GpuTableSet(gpu, [A.Categorical(m) for m in ms])
        cap = ts.slot_capacity(L)
        nch = n // L
        setups.append(dict(ts=ts, cap=cap, slots=torch.empty(nch * cap, dtype=torch.uint8, device="cuda"),
                           lens=torch.zeros(nch, dtype=torch.int32, device="cuda"),
                           status=torch.zeros(1, dtype=torch.int32, device="cuda"), out=torch.empty_like(syms)))

    def step(i, ev):
        A._lib = libs[i]
        s = setups[i]
        ev[0].record(stream)
        s["ts"].dev_encode(d_tids, syms, 1, n, L, s["slots"], s["cap"], s["lens"], s["status"], stream)
        ev[1].record(stream)
        s["ts"].dev_decode(d_tids, s["slots"], None, s["cap"], s["lens"], n, L, s["out"], 1, s["status"], stream)
        ev[2].record(stream)

    for _ in range(3):
        for i in range(2):
            step(i, [torch.cuda.Event(enable_timing=True) for _ in range(3)])
    torch.cuda.synchronize()
    evs = [[], []]
    for it in range(iters):
        for i in ((0, 1) if it % 2 == 0 else (1, 0)):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            step(i, ev)
            evs[i].append(ev)
        if sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    for i in range(2):
        s = setups[i]
        A._lib = libs[i]
        assert s["ts"].gpu.status(s["status"], stream) == 0
        assert torch.equal(s["out"], syms), f"{dirs[i]}: round trip"
        te = np.median([e[0].elapsed_time(e[1]) for e in evs[i]])
        td = np.median([e[1].elapsed_time(e[2]) for e in evs[i]])
        print(f"{dirs[i]:10s} enc {te:.4f} dec {td:.4f} ms (median of {iters})", flush=True)
    # (the slots past each stream's length hold whatever the buffer held: compare the lengths
    # and each stream's own bytes)
    same = torch.equal(setups[0]["lens"], setups[1]["lens"])
    if same:  # every 64th chunk's stream bytes
        cap = setups[0]["cap"]
        lens = setups[0]["lens"].cpu().numpy()
        a = setups[0]["slots"].view(-1, cap)[::64].cpu().numpy()
        b = setups[1]["slots"].view(-1, cap)[::64].cpu().numpy()
        same = all(np.array_equal(a[i, :lens[64 * i]], b[i, :lens[64 * i]]) for i in range(len(a)))
    print("streams: identical" if same else "note: the two builds' streams differ", flush=True)


def main():
    dirs = sys.argv[1:3]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    sync = os.environ.get("AB_NOSYNC") != "1"  # AB_NOSYNC=1: back-to-back launches, no idle gaps
    if os.environ.get("AB_CONFIG") == "indep":
        return indep(dirs, iters, sync)
    masses_name, log2n, sym_bytes, seed = bench.CONFIGS[os.environ.get("AB_CONFIG", "c3")]
    masses_fn = getattr(A, masses_name)
    dense = os.environ.get("AB_DENSE") == "1"
    log2n = int(os.environ.get("AB_LOG2N", log2n))
    n, L = 1 << log2n, 4096
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    libs = [load(d) for d in dirs]
    setups = []
    syms = torch.empty(n, dtype={1: torch.uint8, 2: torch.int16, 4: torch.int32}[sym_bytes], device="cuda")
    for i, Lb in enumerate(libs):
        A._lib = Lb
        gpu = A.Gpu(0)
        gt = A.GpuTable(gpu, A.Categorical(masses_fn()))
        if i == 0:
            gt.dev_gen_iid(seed, 0, n, syms, sym_bytes, stream)
        cap = gt.slot_capacity(L)
        nch = -(-n // L)
        setups.append(dict(gpu=gpu, gt=gt, cap=cap,
                           slots=torch.empty(nch * cap, dtype=torch.uint8, device="cuda"),
                           lens=torch.zeros(nch, dtype=torch.int32, device="cuda"),
                           status=torch.zeros(1, dtype=torch.int32, device="cuda"),
                           out=torch.empty_like(syms),
                           offs=torch.empty(A.dense_offsets_entries(nch), dtype=torch.int64, device="cuda"),
                           dense=torch.empty(nch * cap, dtype=torch.uint8, device="cuda") if dense else None))

    def step(i, ev):
        A._lib = libs[i]
        s = setups[i]
        ev[0].record(stream)
        if dense:
            s["gt"].dev_encode_dense(syms, sym_bytes, n, L, s["slots"], s["cap"], s["lens"], s["offs"], s["dense"],
                                     s["status"], stream)
        else:
            s["gt"].dev_encode(syms, sym_bytes, n, L, s["slots"], s["cap"], s["lens"], s["status"], stream)
        ev[1].record(stream)
        if dense:
            s["gt"].dev_decode(s["dense"], s["offs"], s["cap"], s["lens"], n, L, s["out"], sym_bytes, s["status"], stream)
        else:
            s["gt"].dev_decode(s["slots"], None, s["cap"], s["lens"], n, L, s["out"], sym_bytes, s["status"], stream)
        ev[2].record(stream)

    for _ in range(3):
        for i in range(2):
            step(i, [torch.cuda.Event(enable_timing=True) for _ in range(3)])
    torch.cuda.synchronize()
    evs = [[], []]
    for it in range(iters):
        # the order alternates: after each synchronisation the GPU idles and its clocks drop
        # a little, which otherwise charged ~0.5-1% to whichever build ran first
        for i in ((0, 1) if it % 2 == 0 else (1, 0)):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            step(i, ev)
            evs[i].append(ev)
        if sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    for i in range(2):
        s = setups[i]
        if os.environ.get("AB_NOCHECK") != "1":
            assert torch.equal(s["out"], syms), f"{dirs[i]}: round trip differs"
            assert int(s["status"].item()) == 0, f"{dirs[i]}: device status {int(s['status'].item())}"
        enc = np.median([e[0].elapsed_time(e[1]) for e in evs[i]])
        dec = np.median([e[1].elapsed_time(e[2]) for e in evs[i]])
        print(f"{dirs[i]:10s} enc {enc:.4f} dec {dec:.4f} ms (median of {iters}{'' if sync else ', no sync'})")
        if os.environ.get("AB_TRACE") == "1":
            print(" ".join(f"{e[0].elapsed_time(e[1]):.3f}/{e[1].elapsed_time(e[2]):.3f}" for e in evs[i]))
    if os.environ.get("AB_NOCHECK") != "1":
        assert torch.equal(setups[0]["lens"], setups[1]["lens"]), "the two builds' stream lengths differ"
    sys.stdout.flush()
    # the two builds' table objects would be freed through whichever build is current when main's
    # frame unwinds: skip the teardown (their layouts may differ)
    os._exit(0)


if __name__ == "__main__":
    main()
