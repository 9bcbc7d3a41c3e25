"""Config C1: the reference's `cargo test --release benchmark_multiset -- --ignored`
(src/multiset.rs:155-175), vector part, on this library.

For each fixture multiset-data/{1000,10000,100000}.txt (tests/golden/): the IID<Categorical>
with the reference's table (masses max(1, floor(p * 2^28)), src/multiset.rs:169-170) is run
through Codec::test with TestConfig::test(0)'s initial message Message::random(0)
(src/benchmark.rs:590-595,698-700), printing `bits amortized_bits enc_sec dec_sec` like
test_and_print.  Host coder (ans_core.hpp through the C ABI) first; with a GPU, the C2 layout
too (64 chunks = one wave of chains, Message::zeros() per chunk, device-resident timing).
The "as multiset with shuffle coding" half of the harness is out of scope.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402

import ans_amd as A  # noqa: E402


def main():
    golden = os.path.join(ROOT, "tests", "golden")
    masses = json.load(open(os.path.join(golden, "masses_multiset.json")))["masses"]
    cat = A.Categorical(masses)
    gpu = None
    try:
        if A.device_count() > 0:
            gpu = A.Gpu(0)
    except A.AnsError:
        gpu = None
    rows = []
    for size in (1000, 10000, 100000):
        v = A.read_multiset(os.path.join(golden, f"multiset_{size}.txt"))
        assert len(v) == size
        print(f"vector with {size} elements:")
        res = A.IID(cat, size).test(v, A.Message.random(0))
        print(f"{res.bits} {res.amortized_bits} {res.enc_sec} {res.dec_sec} ")
        row = {"size": size, "bits": res.bits, "amortized_bits": res.amortized_bits, "enc_sec": res.enc_sec,
               "dec_sec": res.dec_sec}
        if gpu is not None:
            import torch
            gt = A.GpuTable(gpu, cat)
            L = -(-size // 64)
            n = size
            s = torch.tensor(np.asarray(v, np.int16), device="cuda")
            cap = gt.slot_capacity(L)
            nch = -(-n // L)
            slots = torch.empty(nch * cap, dtype=torch.uint8, device="cuda")
            lens = torch.zeros(nch, dtype=torch.int32, device="cuda")
            st = torch.zeros(1, dtype=torch.int32, device="cuda")
            back = torch.empty_like(s)
            stream = torch.cuda.Stream()  # a real stream handle (0 would mean the context's own)
            torch.cuda.synchronize()
            te, td = [], []
            for r in range(6):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(stream)
                gt.dev_encode(s, 2, n, L, slots, cap, lens, st, stream)
                ev[1].record(stream)
                gt.dev_decode(slots, None, cap, lens, n, L, back, 2, st, stream)
                ev[2].record(stream)
                torch.cuda.synchronize()
                if r:
                    te.append(ev[0].elapsed_time(ev[1]) / 1e3)
                    td.append(ev[1].elapsed_time(ev[2]) / 1e3)
            assert gpu.status(st, stream) == 0 and torch.equal(back, s)
            row["gpu_c2"] = {"chunk_len": L, "chunks": nch, "bytes": int(lens.sum().item()),
                             "enc_sec": float(np.median(te)), "dec_sec": float(np.median(td))}
            print(f"  GPU, {nch} chunks of {L}: {row['gpu_c2']['bytes']} bytes, "
                  f"enc {row['gpu_c2']['enc_sec']:.3e} s, dec {row['gpu_c2']['dec_sec']:.3e} s")
        rows.append(row)
        print()
    print(json.dumps({"config": "C1 benchmark_multiset (vector part)", "rows": rows}))


if __name__ == "__main__":
    main()
