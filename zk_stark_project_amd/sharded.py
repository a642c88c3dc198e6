"""Coset-sharded proving of one STARK over several ranks.

The prover splits the LDE domain by coset; see DESIGN.md §5 and the
`zkp_prove_sharded` comment in include/zkp.h for the exchange steps. Two ways
to form the rank group:

* `prove_local_group` — ranks as threads of this process, each with its own
  `Context` (on one shared GPU or on several); collectives are device copies.
  This is how the multi-rank path is tested on a one-GPU box.
* `rccl_group_comm` — one process per GPU under torchrun; the library's own
  RCCL communicator (xGMI) carries the collectives, torch.distributed only
  broadcasts the 128-byte RCCL unique id.

Every rank returns the same proof bytes, identical to `Context.prove`'s.
"""
from __future__ import annotations

import threading

from . import _native


def prove_local_group(world: int, air_id: int, trace, pub, options, contexts=None, devices=None):
    """Run one sharded proof with `world` in-process ranks; returns [(bytes, transcript)] per rank."""
    comms = _native.local_group(world)
    if contexts is None:
        devices = devices or [0] * world
        contexts = [_native.Context(devices[r]) for r in range(world)]
    results = [None] * world
    errors = [None] * world

    def run(r):
        try:
            results[r] = contexts[r].prove_sharded(comms[r], air_id, trace, pub, options)
        except Exception as e:  # noqa: BLE001 — re-raised below
            errors[r] = e

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for c in comms:
        c.close()
    for e in errors:
        if e is not None:
            raise e
    return results


def rccl_group_comm(ctx, rank: int, world: int):
    """RCCL communicator for this process's rank; torch.distributed must be initialised."""
    import torch
    import torch.distributed as dist

    buf = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        buf.copy_(torch.frombuffer(bytearray(_native.rccl_unique_id()), dtype=torch.uint8))
    if dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        b = buf.to(dev)
        dist.broadcast(b, 0)
        buf = b.cpu()
    else:
        dist.broadcast(buf, 0)
    return ctx.rccl_comm(bytes(buf.numpy().tobytes()), world, rank)
