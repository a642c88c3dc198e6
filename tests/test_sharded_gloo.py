"""world_size-2 gloo test of the sharded group's host logic (CPU, no GPU):
rccl_group_comm hands rank 0's RCCL unique id to every rank, and every rank
creates its communicator with its own (rank, world). The library calls that
need a device (ncclGetUniqueId, ncclCommInitRank) are stubbed."""
import os

import torch.distributed as dist
import torch.multiprocessing as mp

from test_replicas_gloo import _free_port


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zk_stark_project_amd import _native, sharded
    if rank == 0:
        _native.rccl_unique_id = lambda: bytes((7 * i + 3) % 256 for i in range(128))
    else:  # only rank 0 may create the id; the others must receive it
        def no_id():
            raise AssertionError("non-zero rank asked for an RCCL id")
        _native.rccl_unique_id = no_id

    class FakeCtx:
        def rccl_comm(self, uid, w, r):
            return (uid, w, r)

    uid, w, r = sharded.rccl_group_comm(FakeCtx(), rank, world)
    out[rank] = (uid, w, r)
    dist.destroy_process_group()


def test_two_rank_rccl_id_broadcast_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    want = bytes((7 * i + 3) % 256 for i in range(128))
    for r in range(world):
        uid, w, rr = out[r]
        assert uid == want and w == world and rr == r
