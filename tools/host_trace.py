"""The host-memory leg of the bench (C3 through ans_gpu_encode_chunks / ans_gpu_decode_chunks on
page-locked buffers, bench.py host_pass) alone, for a rocprofv3 --hip-trace --memory-copy-trace
--kernel-trace run: prints each call's wall time.
usage: python tools/host_trace.py [log2n=30] [reps=3]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n, L = 1 << log2n, 4096
    g = A.Gpu(0)
    if os.environ.get("HT_BATCH_MB"):  # pipeline batch size (ans_gpu_set_batch_bytes)
        A._check(A.lib().ans_gpu_set_batch_bytes(g.h, int(os.environ["HT_BATCH_MB"]) << 20), "batch")
    gt = A.GpuTable(g, A.Categorical(A.c3_masses()))
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    gt.dev_gen_iid(1, 0, n, d, 1, None)
    torch.cuda.synchronize()
    nch = n // L
    cap = gt.slot_capacity(L) * nch
    hs = A.pinned_empty(n, np.uint8)
    torch.from_numpy(hs).copy_(d.cpu())
    ho = A.pinned_empty(cap, np.uint8)
    hb = A.pinned_empty(n, np.uint8)
    offs = np.zeros(nch, np.uint64)
    lens = np.zeros(nch, np.uint64)
    total = ctypes.c_uint64(0)
    lib = A.lib()
    for r in range(reps):
        t0 = time.perf_counter()
        A._check(lib.ans_gpu_encode_chunks(gt.h, hs.ctypes.data, 1, n, L, ho.ctypes.data, cap, offs.ctypes.data,
                                           lens.ctypes.data, ctypes.byref(total)), "encode")
        t1 = time.perf_counter()
        A._check(lib.ans_gpu_decode_chunks(gt.h, ho.ctypes.data, total.value, offs.ctypes.data, lens.ctypes.data, n, L,
                                           A.GEN_ZEROS, hb.ctypes.data, 1), "decode")
        t2 = time.perf_counter()
        print(f"rep {r}: encode {1e3 * (t1 - t0):.2f} ms ({n / (t1 - t0) / 2**30:.1f} GiB/s), "
              f"decode {1e3 * (t2 - t1):.2f} ms ({n / (t2 - t1) / 2**30:.1f} GiB/s)", flush=True)
    assert np.array_equal(hb, hs)


if __name__ == "__main__":
    main()
