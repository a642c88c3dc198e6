"""world_size-2 gloo test of the multi-rank bench path (CPU, no GPU)."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zk_stark_project_amd.replicas import aggregate_rate, timed_replicas
    calls = []

    def prove_once():  # stand-in for a proof; rank 1 is slower
        time.sleep(0.02 * (rank + 1))
        calls.append(1)
        return rank

    elapsed, local, res = timed_replicas(prove_once, steps=3, warmup=1, dist=dist)
    out[rank] = (elapsed, local, res, len(calls), aggregate_rate(world, 3, elapsed))
    dist.destroy_process_group()


def test_two_rank_replicas_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    e0, l0, r0, c0, v0 = out[0]
    e1, l1, r1, c1, v1 = out[1]
    assert c0 == c1 == 4 and (r0, r1) == (0, 1)
    assert e0 == e1 == pytest.approx(max(l0, l1))  # max over ranks, identical on all ranks
    assert e0 >= 3 * 0.04
    assert v0 == pytest.approx(2 * 3 / e0)
