"""RCCL (torch.distributed "nccl" on ROCm) on the GPU before the 8-GPU run
needs it: the one collective north_star introduces -- the
all-gather of per-rank {units, routes, digest} records and the MAX of the
elapsed time (openr_amd/shard.py) -- initialised at world size 1 on cuda:0
in this process (env rendezvous on 127.0.0.1), with 64-bit digests at and
above 2^63 (the golden c3 digest b6e9...) that must survive the int64
round trip through the device."""
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_reduce_stats_and_xor():
    import torch
    import torch.distributed as dist

    from openr_amd import shard
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")))
    c3 = int(golden["c3"], 16)
    assert c3 >= 1 << 63  # exercises the sign bit of the int64 carrier
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}",
                            rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        units, routes, dg, el, rows = shard.reduce_stats(dist, torch, dev, 2080, 432_640_000,
                                                         c3 >> 1, 1.25e-3)
        assert (units, routes, dg) == (2080, 432_640_000, c3 >> 1)
        assert el == pytest.approx(1.25e-3)
        assert rows == [[2080, 432_640_000, c3 >> 1, 0]]
        digests = [c3, int(golden["c4"], 16), 0xFFFFFFFFFFFFFFFF, 0]
        assert shard.reduce_xor(dist, torch, dev, digests) == digests
        # a real collective on device memory: the all-gather above ran on
        # cuda:0 tensors (reduce_stats keeps them on `dev` under nccl)
        t = torch.arange(4, dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.tolist() == [0, 1, 2, 3]
    finally:
        dist.destroy_process_group()
