"""bench.py's launch contract (the driver's `python bench.py --gpus N`, one process per GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def test_gpus_must_match_world_size():
    # under a launcher, --gpus must equal WORLD_SIZE (refused before any GPU call)
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_launches_two_ranks_itself():
    """`bench.py --gpus 2` with no launcher starts two ranks (a torch.distributed.run child, no
    exec) that share the box's one GPU with gloo for the barrier and gather: rank 0's line says
    n_gpus 2, the value aggregates both shards, and the C4 sub-object reports both ranks."""
    env = dict(os.environ, BENCH_SHARE_DEVICE="1", BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1", "--log2n", "24",
           "--c4-log2n", "22", "--no-cpu-baseline", "--no-dense", "--no-host"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak"
    # whole-job aggregate: both 2^24-symbol shards over the slowest rank's time per step
    assert abs(d["value"] - 2 * (1 << 24) / (d["ms_per_step"] * 1e-3) / 2**30) < 0.01 * d["value"]
    assert d["per_rank_ms_per_step"]["max"] == d["ms_per_step"]
    assert d["c4"]["per_rank"]["ms_per_step"]["max"] == d["c4"]["ms_per_step"]
    assert d["c4"]["workload"].startswith("C4: 2^22 iid u16 symbols per GPU")
    assert d["config"]["symbols_per_rank"] == [1 << 24, 1 << 24]


def _two_ranks(extra, timeout=110, **env_extra):
    env = dict(os.environ, BENCH_SHARE_DEVICE="1", BENCH_BACKEND="gloo", **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--no-dense", "--no-host"] + extra
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.gpu
def test_bench_strong_scaling_two_ranks():
    """--strong --gpus 2: the config's 2^log2n symbols in total, split into whole-chunk ranges over
    the ranks (shards.shard_symbols); the two shards' symbol counts sum to 2^log2n and the value
    is the whole array over the slowest rank's step."""
    r = _two_ranks(["--strong", "--log2n", "25", "--no-c4"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    per = d["config"]["symbols_per_rank"]
    assert len(per) == 2 and sum(per) == 1 << 25 and all(p % 4096 == 0 for p in per)
    assert d["config"]["symbols_total"] == 1 << 25
    assert abs(d["value"] - (1 << 25) / (d["ms_per_step"] * 1e-3) / 2**30) < 0.01 * d["value"]


@pytest.mark.gpu
def test_bench_failing_rank_ends_every_rank():
    """A rank whose launch raises (the hidden --test-fail-rank flag) must not leave the other rank
    in the timed region's barrier: both reach the same failure agreement and exit non-zero, well
    inside the launcher's own timeouts."""
    r = _two_ranks(["--log2n", "22", "--no-c4", "--test-fail-rank", "1"], timeout=100)
    assert r.returncode != 0
    assert "failed on rank(s) [1]" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.gpu
def test_bench_eight_ranks_one_device():
    """The driver's 8-GPU scaling launch rehearsed on one device: `bench.py --gpus 8` starts eight
    ranks (global symbol offsets 0..7 x 2^20, the same rank order and shard layout as on an 8-GPU
    node), rank 0 prints one JSON line with eight per-rank entries and the C4 sub-object's
    per-rank spread; gloo carries the barrier and the gather (RCCL needs a GPU per rank)."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "8", "--steps", "3", "--warmup", "1", "--log2n", "20",
                        "--c4-log2n", "18", "--no-cpu-baseline", "--no-dense", "--no-host"],
                       env={k: v for k, v in dict(os.environ, BENCH_SHARE_DEVICE="1", BENCH_BACKEND="gloo").items()
                            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")},
                       capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["scaling"] == "weak"
    assert d["config"]["symbols_per_rank"] == [1 << 20] * 8
    assert d["config"]["symbols_total"] == 8 << 20
    assert abs(d["value"] - 8 * (1 << 20) / (d["ms_per_step"] * 1e-3) / 2**30) < 0.01 * d["value"]
    assert d["c4"]["per_rank"]["ms_per_step"]["max"] == d["c4"]["ms_per_step"]
    assert d["c4"]["workload"].startswith("C4: 2^18 iid u16 symbols per GPU (0.00390625 GiB over 8 GPUs)")


def test_c4_l2_share_follows_the_staged_bucket_width():
    # bench.c4_l2_share restates build_fast_table's rule for k_decode_w's LDS buckets: C4 stages
    # 6,016 buckets of width 4,096 (twice the global 2,048), so 18.3% of the cf space minus the
    # 0.23% of it past a staged bucket's five candidates (re-fetched from L2) is served by LDS
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "shuffle-coding_amd"))
    import numpy as np

    import ans_amd as A
    import bench

    m = A.c4_masses()
    norm = int(m.sum())
    share = bench.c4_l2_share(m)
    covered = 6016 * 4096
    assert 1.0 - covered / norm < share < 1.0 - 0.99 * covered / norm
    assert abs(share - 0.8174) < 1e-3
    # a table whose buckets all fit in LDS at the fine width serves every lookup from LDS
    assert bench.c4_l2_share(np.full(300, 20, dtype=np.uint64)) == 0.0  # norm 6,000: 6,000 buckets
