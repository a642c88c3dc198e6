"""zkp_comm_check and the RCCL backend on the one-GPU box.

RCCL refuses two ranks on one device, so the driver's multi-GPU bench is the
first RCCL run with peers. A world-1 RCCL communicator still executes
ncclCommInitRank, the grouped ncclSend/ncclRecv all-to-all and ncclAllGather of
`csrc/comm.cpp` (to itself) through zkp_comm_check's verified exchange, and a
sharded proof over it must equal zkp_prove's bytes."""
import threading

import pytest

from zk_stark_project_amd import AIR_MIMC, MimcProver, ProofOptions, _native
from zk_stark_project_amd.sharded import prove_local_group

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_comm_check_local_group(world):
    comms = _native.local_group(world)
    ctxs = [_native.Context(0) for _ in range(world)]
    out, errs = [None] * world, [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].comm_check(comms[r], 1 << 20)
        except Exception as e:  # noqa: BLE001 — re-raised below
            errs[r] = e
    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert [c.backend_world for c in comms] == [world] * world
    for c in comms:
        c.close()
    assert errs == [None] * world
    assert all(a > 0 and g > 0 for a, g in out)


def test_comm_check_rejects_bad_block(ctx):
    comm = _native.local_group(1)[0]
    with pytest.raises(_native.ZkpError):
        ctx.comm_check(comm, 6)  # not a multiple of 4
    comm.close()


def test_rccl_world1_check_and_proof(ctx):
    comm = ctx.rccl_comm(_native.rccl_unique_id(), 1, 0)
    try:
        assert comm.backend_world == 1  # ncclCommCount
        a2a_ms, ag_ms = ctx.comm_check(comm, 4 << 20)
        assert a2a_ms > 0 and ag_ms > 0
        opts = ProofOptions(8, 8, 0)
        p = MimcProver(opts, ctx)
        trace = p.build_trace(5, 1 << 12)
        pub = p.get_pub_inputs(trace).to_elements()
        single, _ = ctx.prove(AIR_MIMC, trace.data, pub, opts)
        sharded, _ = ctx.prove_sharded(comm, AIR_MIMC, trace.data, pub, opts)
        assert sharded == single
    finally:
        comm.close()


def test_local_group_check_then_prove(ctx):
    """A group that ran the check still proves (the check's buffers are separate)."""
    opts = ProofOptions(8, 8, 0)
    p = MimcProver(opts, ctx)
    trace = p.build_trace(9, 1 << 11)
    pub = p.get_pub_inputs(trace).to_elements()
    single, _ = ctx.prove(AIR_MIMC, trace.data, pub, opts)
    res = prove_local_group(2, AIR_MIMC, trace.data, pub, opts)
    assert all(b == single for b, _ in res)


def test_comm_check_detects_a_corrupting_transport(ctx):
    """A caller transport that flips one byte of an all-gather block must make the
    check fail (naming the peer and word), not pass silently."""
    import ctypes

    def a2a(send, recv, block):
        ctypes.memmove(recv, send, block)  # world 1: block 0 to itself

    def ag(send, recv, nbytes):
        ctypes.memmove(recv, send, nbytes)
        b = (ctypes.c_uint8 * nbytes).from_address(recv)
        b[nbytes // 2] ^= 0x40

    comm = _native.host_comm(0, 1, a2a, ag)
    try:
        with pytest.raises(_native.ZkpError, match="all_gather"):
            ctx.comm_check(comm, 1 << 16)
    finally:
        comm.close()
