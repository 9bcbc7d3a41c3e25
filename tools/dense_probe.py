"""Where the dense container's decode time goes: the C3 decode from (a) the slot layout, (b) the
same slots addressed through an offsets array, (c) the dense container, (d) a container whose
streams start 16-B aligned (each stream padded to 16 B).  HIP events, medians of 20.
usage: python3 tools/dense_probe.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "shuffle-coding_amd")]
import ans_amd as A  # noqa: E402


def main():
    n, L = 1 << 30, 4096
    nch = n // L
    g = A.Gpu(0)
    gt = A.GpuTable(g, A.Categorical(A.c3_masses()))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    syms = torch.empty(n, dtype=torch.uint8, device="cuda")
    gt.dev_gen_iid(1, 0, n, syms, 1, stream)
    cap = gt.slot_capacity(L)
    slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
    lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    offs = torch.empty(A.dense_offsets_entries(nch), dtype=torch.int64, device="cuda")
    dense = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
    gt.dev_encode_dense(syms, 1, n, L, slots, cap, lens, offs, dense, status, stream)
    out = torch.empty_like(syms)
    slot_offs = torch.arange(nch, dtype=torch.int64, device="cuda") * cap
    # (d): streams copied to 16-B aligned starts
    l64 = lens.to(torch.int64)
    pad = (l64 + 15) // 16 * 16
    a16 = torch.zeros(nch, dtype=torch.int64, device="cuda")
    a16[1:] = torch.cumsum(pad, 0)[:-1]
    al = torch.zeros(int(pad.sum().item()) + 256, dtype=torch.uint8, device="cuda")
    ho, hl, ha = offs[:nch].cpu().numpy(), l64.cpu().numpy(), a16.cpu().numpy()
    hd = dense.cpu().numpy()
    ha_buf = np.zeros(al.numel(), np.uint8)
    for c in range(nch):
        ha_buf[ha[c]:ha[c] + hl[c]] = hd[ho[c]:ho[c] + hl[c]]
    al.copy_(torch.from_numpy(ha_buf))
    cases = {"slots": (slots, None), "slots via offsets": (slots, slot_offs), "dense": (dense, offs[:nch]),
             "16-B aligned starts": (al, a16)}
    for name, (buf, o) in cases.items():
        times = []
        for it in range(25):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            gt.dev_decode(buf, o, cap, lens, n, L, out, 1, status, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if it >= 5:
                times.append(e0.elapsed_time(e1))
        ok = torch.equal(out, syms) and g.status(status, stream) == 0
        print(f"{name:22s} decode {np.median(times):.4f} ms  ok={ok}", flush=True)


if __name__ == "__main__":
    main()
