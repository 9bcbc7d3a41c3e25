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


def main():
    dirs = sys.argv[1:3]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    sync = os.environ.get("AB_NOSYNC") != "1"  # AB_NOSYNC=1: back-to-back launches, no idle gaps
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
