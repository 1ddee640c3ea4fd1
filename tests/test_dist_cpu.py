"""Multi-rank path of bench.py on CPU (gloo, world_size 2): the work-table broadcast gives
every rank a disjoint shard of the batch, identical to what rank 0 built."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, batch, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seeds = bench.work_table(rank, world, batch, torch.device("cpu"))
    # max-over-ranks timing reduction, as bench.py does it
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, seeds, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_work_table_broadcast_gloo(world):
    batch = 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict()
    for _ in range(world):
        r, seeds, tmax = q.get(timeout=120)
        got[r] = seeds
        assert tmax == float(world)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allseeds = [s for r in range(world) for s in got[r]]
    assert len(allseeds) == world * batch and len(set(allseeds)) == world * batch
    assert got[0] == list(range(1234, 1234 + batch))
    assert got[1] == list(range(1234 + batch, 1234 + 2 * batch))
