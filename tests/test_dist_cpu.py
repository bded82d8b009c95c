"""N>1 plumbing on CPU: world_size-2 gloo processes exercise the barrier and
the max/sum reductions bench.py uses, and the stripe sharding."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

import bcp_dist


def test_shard_range_covers_everything_once():
    for total in (0, 1, 7, 12500, 125000):
        for world in (1, 2, 3, 8):
            spans = [bcp_dist.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    # config 4: 125,000 stripes over 8 GPUs = 15,625 each
    assert all(b - a == 15625 for a, b in (bcp_dist.shard_range(125000, 8, r) for r in range(8)))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    d = bcp_dist.Dist()
    d.barrier()
    mx = d.max(float(rank + 1) * 1.5)
    sm = d.sum(float(rank + 1))
    ids = d.gather(f"0000:{rank % 1:02x}:00.0")  # two ranks on one device, as bench.py sees them
    d.barrier()
    d.close()
    q.put((rank, mx, sm, tuple(ids)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_gloo_world2_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[:3] for r in res] == [(0, 3.0, 3.0), (1, 3.0, 3.0)]
    assert all(r[3] == ("0000:00:00.0", "0000:00:00.0") for r in res)
