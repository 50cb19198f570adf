"""Multi-rank sharding (gloo, world_size 2 and 3, CPU): scatter with halos, global window
indices (row-0 numerics only on global window 0), gather == single-device result.
The per-rank compute is the CPU oracle injected through ``compute`` (test only); on the
GPU box the same functions run the HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import golden_cases as gc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_compute(local, W, S, ids, first_window, n_windows, base_window, **kw):
    import oracle
    names = {v: k for k, v in oracle.FEATURE_IDS.items()}
    out = oracle.window_features(local.numpy(), W, S, [names[i] for i in ids],
                                 first_window=first_window, n_windows=n_windows,
                                 base_window=base_window, **kw)
    return torch.from_numpy(out)


def _worker(rank, world, port, W, S, C, nwin, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pymhealth_amd.distributed import sharded_features
        import oracle
        n = (nwin - 1) * S + W
        rng = np.random.default_rng(7)
        x = torch.from_numpy((rng.standard_normal((n, C) if C > 1 else n) + 0.3)
                             .astype(np.float32)) if rank == 0 else None
        names = ["mean", "var", "std", "skewness", "kurtosis", "zero_crossings", "peak_count"]
        ids = [oracle.FEATURE_IDS[k] for k in names]
        # non-source ranks hold no record: the slice shape comes from `channels`
        res = sharded_features(x, n, W, S, ids, compute=_oracle_compute, channels=C)
        if rank == 0:
            full = oracle.window_features(x.numpy(), W, S, names)
            q.put(bool(gc.same(res.numpy(), full).all()) and res.shape == full.shape)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,S,C,nwin", [(2, 256, 256, 3, 301), (3, 100, 37, 1, 50),
                                              (2, 1024, 128, 1, 9), (3, 16, 16, 1, 2)])
def test_sharded_equals_single(world, W, S, C, nwin):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, S, C, nwin, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_shard_and_sample_ranges():
    from pymhealth_amd.distributed import sample_range, shard_range
    for nw in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            rs = [shard_range(nw, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == nw
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert sample_range(2, 5, 1024, 128) == (256, 4 * 128 + 1024)
    assert sample_range(3, 3, 10, 5) == (15, 15)


def test_bench_generator_is_keyed_by_global_sample():
    """bench.synth_device: a rank generating only its window shard (first_sample = w0 * S)
    gets exactly the samples of the whole record (counter-based), for
    every signal; the noise is a standard normal."""
    import bench
    for cfg in ("cfg2", "cfg3", "cfg5"):
        c = bench.CONFIGS[cfg]
        full = bench.synth_device(c, 6000, torch.device("cpu"), seed=1234)
        part = bench.synth_device(c, 2500, torch.device("cpu"), seed=1234, first_sample=3000)
        assert torch.equal(part, full[3000:5500]), cfg
        other = bench.synth_device(c, 6000, torch.device("cpu"), seed=99)
        assert not torch.equal(other, full), cfg
    s = torch.arange(200000, dtype=torch.int64)
    e = bench._gauss(s, 7)
    assert abs(float(e.mean())) < 0.01 and abs(float(e.std()) - 1.0) < 0.01
    u = bench._uniform(s, 3)
    assert float(u.min()) >= 0.0 and float(u.max()) < 1.0


def test_bench_indexed_boundaries_host_device_agree():
    """bench.idx_boundaries: the torch (device) and numpy (CPU baseline) forms give the same
    global boundaries, lengths S - 16 .. S + 16, and a rank's shard is the global slice."""
    import bench
    S = 256
    bn = bench.idx_boundaries(0, 5001, S)
    bt = bench.idx_boundaries(0, 0, S, xp=torch.arange(0, 5001, dtype=torch.int64)).numpy()
    assert np.array_equal(bn, bt)
    d = np.diff(bn)
    assert d.min() >= S - bench.IDX_JITTER and d.max() <= S + bench.IDX_JITTER
    assert len(set(d.tolist())) > 4                 # lengths really vary
    assert np.array_equal(bench.idx_boundaries(3000, 101, S), bn[3000:3101])
    assert bn[0] >= 0


BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    """`python bench.py --gpus N` without WORLD_SIZE starts N ranks itself (the driver's
    SCALE command), every rank joins one process group, and rank 0 reports n_gpus = N."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--backend", "gloo",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and sorted(res["ranks"]) == list(range(n))


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_bench_strong_mode_collectives_on_cpu():
    """`bench.py --gpus 2 --backend gloo --strong --config cfg5 --windows 20000` (here with
    the CPU hook --dry-run: host tensors, no feature compute): two ranks, the record on rank
    0 scattered with its (W - S) halos, rows gathered back; the JSON line reports strong
    scaling with the scatter / compute / gather phase times and byte counts."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--strong",
                        "--config", "cfg5", "--windows", "20000", "--steps", "2", "--warmup", "1",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong"
    assert res["config"]["windows_total"] == 20000 and res["config"]["backend"] == "gloo"
    ph = res["phases"]
    assert ph["scatter_ms"] > 0 and ph["gather_ms"] > 0 and ph["compute_ms"] >= 0
    # rank 1's windows 10000 .. 19999 need samples [10000 * 128, 19999 * 128 + 1024)
    assert ph["scatter_bytes_from_rank0"] == 4 * ((19999 * 128 + 1024) - 10000 * 128)
    assert ph["gather_bytes_to_rank0"] == 10000 * 2 * 8
    assert res["value"] > 0 and "dry_run" in res
