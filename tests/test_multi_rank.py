"""World-size-2 gloo tests of the multi-GPU path on CPU:
every unit is solved by exactly one rank, and the all-gathered per-rank
{units, routes, digest} records reproduce the single-process job. Route
databases come from the CPU oracle here (the GPU product is covered by the
-m gpu parity tests); what is under test is the sharding + reduction code
bench.py runs on the GPU box."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openr_amd import shard

GRID = dict(n=6, metricSeed=0xC2000000, prefixSeed=0xC1)
TOPOS = 10  # whole job


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _route_counts(dbs):
    return sum(db.count(b"\n") for db in dbs)


def _job_stats(oracle, lo, hi):
    dbs = oracle.grid_batch_route_dbs(GRID, lo, hi, "1", False)
    return hi - lo, _route_counts(dbs), shard.route_digest(*[bytearray(d) for d in dbs])


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _refcpu
        lo, hi = shard.block_range(TOPOS, rank, world)
        units, routes, digest = _job_stats(_refcpu, lo, hi)
        res = shard.reduce_stats(dist, torch, torch.device("cpu"), units, routes, digest,
                                 0.5 + rank)
        fabric = shard.interleave([f"n{i}" for i in range(11)], rank, world)
        gathered = [None] * world
        dist.all_gather_object(gathered, fabric)
        out_q.put((rank, res, gathered, (lo, hi)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    results.sort(key=lambda x: x[0])
    # every rank sees the same reduced record
    assert results[0][1][:4] == results[1][1][:4]
    total_units, total_routes, digest, tmax, rows = results[0][1]
    assert tmax == 1.5  # MAX over ranks
    # blocks tile the job exactly once
    assert [r[3] for r in results] == [(0, 5), (5, 10)]
    # the gathered job equals the single-process job, rank by rank
    expect = [_job_stats(oracle, lo, hi) for lo, hi in [(0, 5), (5, 10)]]
    assert total_units == TOPOS
    assert total_routes == sum(e[1] for e in expect)
    assert digest == shard.combine_digests(e[2] for e in expect)
    assert [tuple(r[:3]) for r in rows] == [tuple(e) for e in expect]
    # C3-style interleave covers every source exactly once
    got = sorted(x for part in results[0][2] for x in part)
    assert got == sorted(f"n{i}" for i in range(11))


@pytest.mark.parametrize("total,world", [(4096, 1), (4096, 8), (10, 3), (2, 4), (0, 2)])
def test_block_range_tiles(total, world):
    seen = []
    for r in range(world):
        lo, hi = shard.block_range(total, r, world)
        assert 0 <= lo <= hi <= total
        seen.extend(range(lo, hi))
    assert seen == list(range(total))


def test_bad_rank_rejected():
    with pytest.raises(ValueError):
        shard.block_range(10, 2, 2)
    with pytest.raises(ValueError):
        shard.interleave([1, 2], -1, 2)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_unit_digest_independent_of_sharding(world):
    """bench.py's job digest (XOR of per-unit keyed hashes) is the same
    whether the units are solved on one rank or split over `world` ranks,
    block-wise or interleaved."""
    import numpy as np
    rng = np.random.default_rng(7)
    U = 37
    meta = rng.integers(0, 2**31, size=(U, 16), dtype=np.int32)
    mask = rng.integers(0, 2**31, size=(U, 2, 16), dtype=np.int32)
    keys = list(range(U))
    whole = shard.unit_digest(keys, meta, mask)
    blocks = []
    for r in range(world):
        lo, hi = shard.block_range(U, r, world)
        blocks.append(shard.unit_digest(keys[lo:hi], meta[lo:hi], mask[lo:hi]))
    assert shard.combine_digests(blocks) == whole
    inter = [shard.unit_digest(shard.interleave(keys, r, world),
                               meta[r::world], mask[r::world]) for r in range(world)]
    assert shard.combine_digests(inter) == whole
    flipped = meta.copy()
    flipped[5, 3] ^= 1
    assert shard.unit_digest(keys, flipped, mask) != whole


# ------------------------------------------------ bench.py --gpus N launcher --
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _bench(args, env_extra=None, timeout=280):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.timeout(300)
def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher around it starts two ranks itself
    (children, gloo here), and a WORLD_SIZE that disagrees with --gpus is an
    error, never a silent N=1 run."""
    rc, line, err = _bench(["--gpus", "2", "--launch-check"])
    assert rc == 0, err[-2000:]
    assert line == {"world": 2, "ranks": [[0, 0], [1, 1]]}
    rc, line, _ = _bench(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1"})
    assert rc == 2 and line is None


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_share_device_golden():
    """The N=2 path end to end on one GPU (OGS_BENCH_SHARE_DEVICE=1: both
    ranks on device 0, gloo for the records): `--gpus 2` launches the ranks,
    and the C2 (weak: blocks 0+1) and C3 (strong: interleaved sources) job
    digests equal the oracle's golden values at N=2."""
    share = {"OGS_BENCH_SHARE_DEVICE": "1"}
    rc, line, err = _bench(["--gpus", "2", "--config", "c2", "--steps", "3", "--warmup", "1",
                            "--no-cpu-baseline"], share)
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 2 and line["golden"]["c2"] == "match"
    assert line["config"]["topologies_per_gpu"] == 4096
    rc, line, err = _bench(["--gpus", "2", "--config", "c3", "--steps", "2", "--warmup", "1",
                            "--no-cpu-baseline", "--no-extras"], share)
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 2 and line["golden"]["c3"] == "match"
