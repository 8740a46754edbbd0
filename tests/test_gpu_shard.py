"""GPU, world_size 2 (gloo): the multi-GPU path with libecamd doing the work in every rank.

Two rank processes (fresh interpreters, as bench.py starts them) share the box's GPU: each encodes
its own shard of stripes with ecamd_rs_encode, checks the parity of every stripe it owns against
the CPU oracle, and the ranks all-reduce a digest of their shards and the stripe count over gloo.
The reduced digest equals the one a single process computes from the oracle over the whole batch,
so the shards cover every stripe exactly once and each was encoded correctly on the device.
Reference: stripes are independent (src/erasurecode.c:383-477), so ranks need no data exchange.
"""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

K, M, BS, PER_RANK = 4, 2, 65536 + 16, 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(data, parity):
    return int(hashlib.sha256(data.tobytes() + parity.tobytes()).hexdigest()[:12], 16)


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import oracle_lib as orc
    from ecdata import stripe_fragments
    from liberasurecode_amd import device as D
    from liberasurecode_amd.shard import Coordinator, stripe_range
    co = Coordinator(backend="gloo")
    try:
        first, n = stripe_range(co.rank, co.world, PER_RANK)
        lay = D.Layout.alloc(K + M, BS, n)
        lay.fill_splitmix(nfrags=K, stripe0=first)
        D.rs_encode(K, M, lay)
        got = lay.download_stripes()
        lay.buf.free()
        digest, bad = 0, 0
        for i in range(n):
            data = stripe_fragments(first + i, K, BS)
            bad += int(not (got[i, :K] == data).all())
            bad += int(not (got[i, K:] == orc.encode(K, M, data)).all())
            digest += _digest(got[i, :K], got[i, K:])
        co.barrier()
        # 48-bit digests: sums over both shards stay exact in float64 (< 2^53)
        total, count, errors = co.reduce([float(digest), float(n), float(bad)], op="sum")
        q.put((rank, first, n, int(total), int(count), int(errors)))
    finally:
        co.close()


def test_two_ranks_encode_their_shards_on_the_gpu():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import oracle_lib as orc
    from ecdata import stripe_fragments
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
    single = 0
    for s in range(world * PER_RANK):
        data = stripe_fragments(s, K, BS)
        single += _digest(data, orc.encode(K, M, data))
    for rank, first, n, total, count, errors in res:
        assert (first, n) == (rank * PER_RANK, PER_RANK)
        assert errors == 0
        assert count == world * PER_RANK
        assert total == single
