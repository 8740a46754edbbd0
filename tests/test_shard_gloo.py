"""CPU, world_size 2 (gloo): the multi-GPU path's sharding and coordination.  Each rank encodes
its own shard of stripes (with the CPU oracle standing in for the GPU), the shards together cover
every stripe exactly once, and the reduced checksum / elapsed time equal the single-process ones."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

from liberasurecode_amd.shard import split_range, stripe_range

K, M, BS, PER_RANK = 4, 2, 512, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stripe_digest(s):
    import oracle_lib as orc
    from ecdata import stripe_fragments
    data = stripe_fragments(s, K, BS)
    par = orc.encode(K, M, data)
    return int(hashlib.sha256(data.tobytes() + par.tobytes()).hexdigest()[:12], 16)


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from liberasurecode_amd.shard import Coordinator, stripe_range
    co = Coordinator(backend="gloo")
    co.barrier()
    first, n = stripe_range(co.rank, co.world, PER_RANK)
    digest = sum(_stripe_digest(s) for s in range(first, first + n)) % (1 << 50)
    total, count = co.reduce([float(digest), float(n)], op="sum")
    slowest = co.reduce([0.5 + rank], op="max")[0]
    co.close()
    q.put((rank, first, n, int(total), int(count), slowest))


def test_stripe_ranges_partition():
    for world in (1, 2, 3, 8):
        seen = []
        for r in range(world):
            f, n = stripe_range(r, world, 5)
            seen += list(range(f, f + n))
        assert seen == list(range(5 * world))
        seen = []
        for r in range(world):
            f, n = split_range(r, world, 19)
            seen += list(range(f, f + n))
        assert seen == list(range(19))
    with pytest.raises(ValueError):
        stripe_range(2, 2, 1)


def test_two_rank_gloo_shards_cover_everything():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = sum(_stripe_digest(s) for s in range(world * PER_RANK)) % (1 << 50)
    for rank, first, n, total, count, slowest in res:
        assert (first, n) == (rank * PER_RANK, PER_RANK)
        assert total == single % (1 << 50) or total % (1 << 50) == single
        assert count == world * PER_RANK
        assert slowest == 0.5 + world - 1
