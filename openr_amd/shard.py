"""Multi-GPU sharding of SPF + RouteDb batches.

The batch shards embarrassingly: topologies (C2), sources (C3), link-failure
variants (C4) and destinations (C5) are independent units, so every rank
solves its own block with NO data-path collective. The only collectives are
one all-gather of per-rank {units, routes, digest} records and one MAX
all-reduce of the elapsed time (RCCL over xGMI on the GPU box; gloo in the
CPU tests). Nothing here touches a device: the helpers take whatever
process group `torch.distributed` was initialised with.
"""
import hashlib

DIGEST_FIELDS = 4  # units, routes, digest (63-bit), reserved


def block_range(total, rank, world):
    """Contiguous block [lo, hi) of ceil(total / world) units for `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    per = -(-total // world)
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def interleave(items, rank, world):
    """Round-robin share of `items` (C3: balances RSW/FSW/SSW degree classes
    over ranks)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return list(items)[rank::world]


def route_digest(*arrays):
    """63-bit digest of a rank's route records (numpy arrays, in order)."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(memoryview(a).cast("B"))
    return int.from_bytes(h.digest()[:8], "little") >> 1


def unit_digest(keys, *arrays):
    """63-bit digest of a set of units that does not depend on how the units
    are split over ranks: XOR over units of sha256(key, the unit's rows).
    `keys` are global unit ids (ints or strings); every array's leading
    dimension is split into len(keys) equal rows, one per unit."""
    import numpy as np
    n = len(keys)
    rows = [np.ascontiguousarray(a).reshape(n, -1) if n else a for a in arrays]
    out = 0
    for i, k in enumerate(keys):
        h = hashlib.sha256(str(k).encode() + b"\0")
        for r in rows:
            h.update(memoryview(r[i]).cast("B"))
        out ^= int.from_bytes(h.digest()[:8], "little") >> 1
    return out


def combine_digests(digests):
    """Order-independent combination of per-rank digests: XOR (each rank's
    block is fixed by its rank, so XOR of the blocks is the whole job's)."""
    out = 0
    for d in digests:
        out ^= int(d)
    return out


def reduce_stats(dist, torch, device, units, routes, digest, elapsed_s):
    """All-gather per-rank {units, routes, digest}, MAX-reduce elapsed.
    Returns (total_units, total_routes, combined_digest, max_elapsed_s,
    per_rank list). With dist None (single process) it returns the inputs.
    Under gloo (CPU tests, shared-device rehearsal) the records stay on the
    host."""
    if dist is not None and dist.get_backend() == "gloo":
        device = "cpu"
    local = torch.tensor([int(units), int(routes), int(digest), 0],
                         dtype=torch.int64, device=device)
    elapsed = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    if dist is None:
        rows = [local.tolist()]
    else:
        gathered = [torch.zeros_like(local) for _ in range(dist.get_world_size())]
        dist.all_gather(gathered, local)
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        rows = [g.tolist() for g in gathered]
    return (sum(r[0] for r in rows), sum(r[1] for r in rows),
            combine_digests(r[2] for r in rows), float(elapsed.item()), rows)


def _h63(b):
    return int.from_bytes(hashlib.sha256(b).digest()[:8], "little") >> 1


def changes_digest(keys, changes):
    """Config C4 job digest, independent of how variants are split over
    ranks: XOR over variants of a hash of (global variant index, #routes to
    update, #routes to delete, sorted changed prefixes) -- the
    DecisionRouteUpdate key sets of calculateUpdate (SpfSolver.cpp:21-56).
    `changes[i]` = (upd, del, prefixes) of variant keys[i]."""
    out = 0
    for k, (upd, dele, prefixes) in zip(keys, changes):
        out ^= _h63(f"{k}\0{upd}\0{dele}\0".encode() +
                    "\0".join(sorted(prefixes)).encode())
    return out


def lines_digest(lines):
    """XOR of per-line hashes (config C5 KSP2 path lines "area dest k:...",
    one per (destination, k)): independent of destination order and of the
    destination blocks the ranks own."""
    out = 0
    for ln in lines:
        out ^= _h63(ln.encode() if isinstance(ln, str) else bytes(ln))
    return out


def _to_i64(d):
    d = int(d) & 0xFFFFFFFFFFFFFFFF
    return d - (1 << 64) if d >= (1 << 63) else d


def reduce_xor(dist, torch, device, digests):
    """XOR-combine a list of 64-bit digests over all ranks (one all-gather);
    with dist None the inputs are returned. The route digests of
    route_digest.h are XOR-decomposable over units / prefixes, so the result
    is the whole job's digest whatever the split."""
    if dist is None:
        return [int(d) & 0xFFFFFFFFFFFFFFFF for d in digests]
    if dist.get_backend() == "gloo":
        device = "cpu"
    local = torch.tensor([_to_i64(d) for d in digests], dtype=torch.int64, device=device)
    gathered = [torch.zeros_like(local) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, local)
    out = [0] * len(digests)
    for g in gathered:
        for i, v in enumerate(g.tolist()):
            out[i] ^= int(v) & 0xFFFFFFFFFFFFFFFF
    return out
