"""The coset-sharded protocol across processes (GPU box): two processes, each
with its own zkp_ctx on device 0, run zkp_prove_sharded with the collectives
carried by torch.distributed/gloo through the library's caller-transport
backend (zkp_comm_host_create). Every rank must return the single-GPU proof
bytes (and so the oracle's). This exercises the multi-process ordering, buffer
lifetimes and abort path that the in-process group cannot; RCCL itself refuses
two ranks on one device, and differs only in the send/recv calls."""
import multiprocessing
import os
import traceback

import pytest

import oracle_ref as O
from test_gpu_parity import gu_prover, mimc_case
from test_replicas_gloo import _free_port
from zk_stark_project_amd import AIR_GLOBAL_UPDATE, AIR_MIMC, ProofOptions
from zk_stark_project_amd.field import to_bytes

pytestmark = pytest.mark.gpu


def _case(kind):
    if kind == "mimc":
        opts = ProofOptions(40, 8, 12)
        p, trace = mimc_case(1 << 13, opts)
        return AIR_MIMC, trace, p.get_pub_inputs(trace).to_elements(), opts
    if kind == "mimc_b16":
        opts = ProofOptions(30, 16, 8)
        p, trace = mimc_case(1 << 12, opts)
        return AIR_MIMC, trace, p.get_pub_inputs(trace).to_elements(), opts
    opts = ProofOptions.reference()
    p = gu_prover(16, 1 << 13, opts, seed=21)
    trace = p.build_trace()
    if kind == "global_update_dev_bad":  # a failed transition on rank 1's rows: both ranks fall back, unpaired
        trace.data[70, (1 << 12) + 9, 0] ^= 0x77
    return AIR_GLOBAL_UPDATE, trace, p.get_pub_inputs(trace).to_elements(), opts


def _rank(rank, world, port, kind, q, fail_rank):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        import datetime
        # a peer that leaves makes the collectives fail instead of blocking for gloo's default 30 min
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
        from zk_stark_project_amd import _native
        from zk_stark_project_amd.sharded import gloo_group_comm
        air, trace, pub, opts = _case(kind)
        ctx = _native.Context(0)
        comm = gloo_group_comm(rank, world)
        if rank == fail_rank:  # this rank fails its argument checks: the peers must not hang
            comm.close()
            q.put((rank, "failed-as-asked", None))
            dist.destroy_process_group()
            return
        try:
            if kind.startswith("global_update_dev"):  # device-resident: the paired path, flags over gloo
                w, n = trace.data.shape[0], trace.data.shape[1]
                d = ctx.alloc(trace.data.nbytes)
                ctx.to_device(d, trace.data)
                data, _ = ctx.prove_sharded(comm, air, d, pub, opts, shape=(w, n))
                ctx.free(d)
            else:
                data, _ = ctx.prove_sharded(comm, air, trace.data, pub, opts)
            q.put((rank, "ok", data))
        except Exception as e:  # noqa: BLE001
            q.put((rank, "error", repr(e)))
        comm.close()
        ctx.close()
        if dist.is_initialized():  # a failed proof already tore the group down (gloo_abort)
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, "crash", traceback.format_exc()))


def run_group(kind, world=2, fail_rank=-1, timeout=240):
    mpc = multiprocessing.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_rank, args=(r, world, port, kind, q, fail_rank)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, status, data = q.get(timeout=timeout)
            res[r] = (status, data)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("kind", ["mimc", "mimc_b16", "global_update", "global_update_dev", "global_update_dev_bad"])
def test_two_process_gloo_sharded_equals_single(ctx, kind):
    air, trace, pub, opts = _case(kind)
    single, _ = ctx.prove(air, trace.data, pub, opts)
    res = run_group(kind)
    for r in range(2):
        status, data = res[r]
        assert status == "ok", f"rank {r}: {status} {data}"
        assert data == single, f"rank {r} bytes differ from the single-GPU proof"
    w, n = trace.data.shape[0], trace.data.shape[1]
    ref, _ = O.prove(air, trace.to_bytes(), w, n, to_bytes(pub), opts)
    assert single == ref


def test_peer_failure_does_not_hang(ctx):
    """Rank 1 leaves before proving: rank 0's first collective fails (the caller
    transport returns an error), zkp_prove_sharded returns ZKP_ERR_DEVICE."""
    res = run_group("mimc", fail_rank=1, timeout=180)
    assert res[1][0] == "failed-as-asked"
    status, data = res[0]
    assert status == "error" and "zkp error 5" in data, (status, data)
