"""Host-memory (PCIe-inclusive) rate of the bulk path on C3.

Times ans_gpu_encode_chunks / ans_gpu_decode_chunks, whose inputs and outputs are host
buffers (H2D copy, kernels, D2H copy), with pageable numpy buffers and with pinned buffers.
Symbols are the C3 workload (counter-based generator), produced on the device
and copied to the host once before timing.  Prints one JSON line.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402


def run(gt, syms_ptr, n, L, out_ptr, out_cap, offs, lens, back_ptr, reps):
    lib = A.lib()
    total = ctypes.c_uint64(0)
    te, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        A._check(lib.ans_gpu_encode_chunks(gt.h, syms_ptr, 1, n, L, out_ptr, out_cap, offs.ctypes.data, lens.ctypes.data,
                                           ctypes.byref(total)), "encode")
        t1 = time.perf_counter()
        A._check(lib.ans_gpu_decode_chunks(gt.h, out_ptr, total.value, offs.ctypes.data, lens.ctypes.data, n, L,
                                           A.GEN_ZEROS, back_ptr, 1), "decode")
        t2 = time.perf_counter()
        te.append(t1 - t0)
        td.append(t2 - t1)
    return min(te), min(td), total.value


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    batch_mib = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # 0 = the library default
    n, L = 1 << log2n, 4096
    masses = A.c3_masses()
    g = A.Gpu(0)
    g.set_batch_bytes(batch_mib << 20)
    gt = A.GpuTable(g, A.Categorical(masses))
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    gt.dev_gen_iid(1, 0, n, d, 1, None)
    torch.cuda.synchronize()
    nch = n // L
    cap = gt.slot_capacity(L) * nch
    res = {"workload": f"C3 2^{log2n} u8 symbols, chunk {L}", "reps": reps, "batch_mib": batch_mib or 256}
    offs = np.zeros(nch, np.uint64)
    lens = np.zeros(nch, np.uint64)
    # pageable numpy buffers
    syms = d.cpu().numpy()
    out = np.empty(cap, np.uint8)
    back = np.empty(n, np.uint8)
    te, td, total = run(gt, syms.ctypes.data, n, L, out.ctypes.data, cap, offs, lens, back.ctypes.data, reps)
    assert np.array_equal(back, syms)
    res["pageable"] = {"encode_gib_s": n / te / 2**30, "decode_gib_s": n / td / 2**30,
                       "round_trip_gib_s": n / (te + td) / 2**30}
    # page-locked buffers from the library (ans_host_alloc)
    hs = A.pinned_empty(n, np.uint8)
    hs[:] = syms
    ho = A.pinned_empty(cap, np.uint8)
    hb = A.pinned_empty(n, np.uint8)
    te, td, total = run(gt, hs.ctypes.data, n, L, ho.ctypes.data, cap, offs, lens, hb.ctypes.data, reps)
    assert np.array_equal(hb, syms)
    res["pinned"] = {"encode_gib_s": n / te / 2**30, "decode_gib_s": n / td / 2**30,
                     "round_trip_gib_s": n / (te + td) / 2**30}
    del hs, ho, hb
    # torch's pinned buffers
    ps = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    ps.copy_(d.cpu())
    po = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    pb = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    te, td, total = run(gt, ps.data_ptr(), n, L, po.data_ptr(), cap, offs, lens, pb.data_ptr(), reps)
    assert torch.equal(pb, ps)
    res["torch_pinned"] = {"encode_gib_s": n / te / 2**30, "decode_gib_s": n / td / 2**30,
                           "round_trip_gib_s": n / (te + td) / 2**30}
    res["compressed_bytes_per_symbol"] = total / n
    print(json.dumps(res))


if __name__ == "__main__":
    main()
