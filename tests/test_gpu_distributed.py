"""The multi-GPU path on the GPU box: ``distributed.sharded_features`` (scatter ->
per-rank fused launch -> gather) under the RCCL backend ("nccl" on ROCm). The box has
one GPU, so the process group has one rank: RCCL's gather runs on hardware and the
result must equal one direct engine launch bit for bit. (World sizes 2 and 3 are covered
with gloo on the CPU, tests/test_distributed.py; bench.py --gpus N runs the N-rank
RCCL gather on a whole node.)"""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_features_under_rccl_world1():
    import torch.distributed as dist
    import bench
    from pymhealth_amd import distributed as D
    from pymhealth_amd.engine import window_features
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        for cfg in ("cfg2", "cfg5"):
            c = bench.CONFIGS[cfg]
            W, S, nw = c["W"], c["S"], 20000
            n = (nw - 1) * S + W
            x = bench.synth_device(c, n, dev, seed=5)
            ids = [bench.FEATURE_IDS[f] for f in c["feats"]]
            kw = dict(fs=c["fs"], band=c["band"], dom=c["dom"])
            got = D.sharded_features(x, n, W, S, ids, device=dev, **kw)
            ref = window_features(x, W, S, ids, **kw)
            torch.cuda.synchronize()
            assert got.shape == ref.shape and torch.equal(got, ref), cfg
            # a shard generated on its own (what rank r of bench.py does) == that slice
            w0 = 7777
            xs = bench.synth_device(c, (nw - w0 - 1) * S + W, dev, seed=5, first_sample=w0 * S)
            part = window_features(xs, W, S, ids, first_window=w0, n_windows=nw - w0,
                                   base_window=w0, **kw)
            assert torch.equal(part, ref[:, :, w0:]), cfg
    finally:
        dist.destroy_process_group()
