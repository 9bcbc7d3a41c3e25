"""Debug: C3-shaped encode/decode on the GPU, report which chunks fail to round-trip."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402

log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
L = 4096
n = 1 << log2n
masses = A.c3_masses()
gpu = A.Gpu(0)
gt = A.GpuTable(gpu, A.Categorical(masses))
cap = gt.slot_capacity(L)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
syms = torch.empty(n, dtype=torch.uint8, device="cuda")
gt.dev_gen_iid(1, 0, n, syms, 1, stream)
nch = n // L
slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
status = torch.zeros(1, dtype=torch.int32, device="cuda")
out = torch.zeros_like(syms)
gt.dev_encode(syms, 1, n, L, slots, cap, lens, status, stream)
torch.cuda.synchronize()
print("encode status", gpu.status(status, stream))
status.zero_()
gt.dev_decode(slots, None, cap, lens, n, L, out, 1, status, stream)
torch.cuda.synchronize()
print("decode status", gpu.status(status, stream))
bad = (out.view(nch, L) != syms.view(nch, L))
badc = torch.nonzero(bad.any(dim=1)).flatten().cpu().numpy()
print("bad chunks", len(badc), "of", nch)
if len(badc):
    print("first", badc[:20], "mod 1024 hist", np.bincount(badc % 1024 // 128, minlength=8))
    c = int(badc[0])
    pos = torch.nonzero(bad[c]).flatten().cpu().numpy()
    print("chunk", c, "len", int(lens[c]), "first bad symbol", pos[:10], "count", len(pos))
