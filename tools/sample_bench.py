"""Device-resident throughput of bulk Codec::samples (ans_dev_sample_iid) on C3's table:
2^30 u8 samples in chunks of 4096 (chunk c = samples(4096, seed + c)).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ans_amd as A  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    L, n = 4096, 1 << log2n
    gt = A.GpuTable(A.Gpu(0), A.Categorical(A.c3_masses()))
    stream = torch.cuda.Stream()
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    ts = []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        gt.dev_sample(7, n, L, out, 1, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1) / 1e3)
    t = float(np.median(ts))
    print(json.dumps({"workload": f"Codec::samples bulk, C3 table, 2^{log2n} u8 samples, chunk {L}",
                      "ms": round(1e3 * t, 4), "gsamples_s": n / t / 1e9, "gib_s": n / t / 2**30}))


if __name__ == "__main__":
    main()
