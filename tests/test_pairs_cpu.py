"""C5 pair sharding (sonar/pairs.py) on CPU: contiguous pair ranges cover every pair once, and
the record all-gather over gloo (world size 2 and 3) reassembles them in pair order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from sonar import pairs


def test_pair_ranges_partition():
    for P in (1, 7, 1000):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                a, b = pairs.pair_range(P, world, r)
                got.extend(range(a, b))
            assert got == list(range(P))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, P, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    a, b = pairs.pair_range(P, world, rank)
    counts = [pairs.pair_range(P, world, g)[1] - pairs.pair_range(P, world, g)[0] for g in range(world)]
    local = torch.tensor([[k * 10.0 + j for j in range(len(pairs.RECORD_FIELDS))] for k in range(a, b)],
                         dtype=torch.float64).reshape(b - a, len(pairs.RECORD_FIELDS))
    allrec = pairs.gather_records(local, world, counts)
    if rank == 0:
        q.put(allrec.numpy())
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 7), (3, 10), (2, 1)])
def test_record_allgather_gloo(world, P):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    exp = np.array([[k * 10.0 + j for j in range(len(pairs.RECORD_FIELDS))] for k in range(P)])
    assert np.array_equal(out, exp)
