"""Multi-GPU driver for `bench.py --gpus N`: one process per GPU, each proving
its own independent trace ("replicas", weak scaling). The proving path has no
data-path collective; torch.distributed is used only for the start/stop
barriers and the max-over-ranks reduction of the wall time.
"""
from __future__ import annotations

import gc
import time


def timed_replicas(prove_once, steps: int, warmup: int, dist=None, device_sync=None, device=None, times=None):
    """Run `warmup` untimed and `steps` timed calls of prove_once() on this rank.

    Timed region: barrier + device sync on both sides. Returns
    (max_elapsed_over_ranks, local_elapsed, last_result). `times`: a list that
    receives each timed call's own wall time in seconds (prove_once returns
    host bytes, so a call ends when its proof is on the host)."""
    result = None
    for _ in range(warmup):
        result = prove_once()
    if dist is not None:
        dist.barrier()
    if device_sync is not None:
        device_sync()
    # no Python garbage collection inside the timed region (the steps allocate only
    # their proof bytes; a collection pass would land in one step's time)
    gc_was_on = gc.isenabled()
    gc.disable()
    try:
        t0 = time.perf_counter()
        for _ in range(steps):
            t1 = time.perf_counter()
            result = prove_once()
            if times is not None:
                times.append(time.perf_counter() - t1)
        if device_sync is not None:
            device_sync()
    finally:
        if gc_was_on:
            gc.enable()
    if dist is not None:
        dist.barrier()
    local = time.perf_counter() - t0
    elapsed = local
    if dist is not None:
        import torch
        t = torch.tensor([local], dtype=torch.float64, device=device if device is not None else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, local, result


def aggregate_rate(world: int, steps: int, elapsed: float) -> float:
    """Whole-job proofs/s: every rank proved `steps` proofs within `elapsed`."""
    return world * steps / elapsed
