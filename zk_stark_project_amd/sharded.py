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
* `gloo_group_comm` — one process per rank, the collectives carried by
  torch.distributed (gloo, host memory) through the library's caller-transport
  backend (`zkp_comm_host_create`): the same exchange points as RCCL, usable
  where RCCL is not (several ranks on one GPU, CPU-side transports).

Every rank returns the same proof bytes, identical to `Context.prove`'s.
"""
from __future__ import annotations

import ctypes
import threading

from . import _native


def prove_local_group(world: int, air_id: int, trace, pub, options, contexts=None, devices=None, shape=None):
    """Run one sharded proof with `world` in-process ranks; returns [(bytes, transcript)] per rank.
    `trace` is a host array, or (shape=(width, n)) a device pointer every rank can read."""
    comms = _native.local_group(world)
    if contexts is None:
        devices = devices or [0] * world
        contexts = [_native.Context(devices[r]) for r in range(world)]
    results = [None] * world
    errors = [None] * world

    def run(r):
        try:
            results[r] = contexts[r].prove_sharded(comms[r], air_id, trace, pub, options, shape=shape)
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


def host_views(send: int, recv: int, send_bytes: int, recv_bytes: int):
    """torch uint8 tensors viewing the library's pinned staging buffers (no copies)."""
    import torch
    sv = torch.frombuffer((ctypes.c_uint8 * send_bytes).from_address(send), dtype=torch.uint8) if send_bytes else \
        torch.empty(0, dtype=torch.uint8)
    rv = torch.frombuffer((ctypes.c_uint8 * recv_bytes).from_address(recv), dtype=torch.uint8) if recv_bytes else \
        torch.empty(0, dtype=torch.uint8)
    return sv, rv


def gloo_transport(world: int, group=None):
    """(all_to_all, all_gather) over torch.distributed on host memory (gloo)."""
    import torch.distributed as dist

    def all_to_all(send, recv, block):
        sv, rv = host_views(send, recv, world * block, world * block)
        if block:
            dist.all_to_all_single(rv, sv, group=group)

    def all_gather(send, recv, nbytes):
        sv, rv = host_views(send, recv, nbytes, world * nbytes)
        if nbytes:
            dist.all_gather_into_tensor(rv, sv, group=group)
    return all_to_all, all_gather


def gloo_abort(group=None):
    """The transport's abort (zkp_comm abort, called by a rank whose proof fails):
    tearing down this rank's process group closes its gloo connections, so peers
    blocked in a collective with it fail at once instead of waiting out the
    group timeout (30 min by default; callers should still init with a short one)."""
    import torch.distributed as dist

    def abort():
        if dist.is_initialized():
            dist.destroy_process_group(group)
    return abort


def gloo_group_comm(rank: int, world: int, group=None):
    """`zkp_comm` whose collectives run over torch.distributed (initialised with gloo).
    On a failed proof the library calls the abort: this rank's group is destroyed
    (check `torch.distributed.is_initialized()` before destroying it again)."""
    a2a, ag = gloo_transport(world, group)
    return _native.host_comm(rank, world, a2a, ag, abort=gloo_abort(group))
