"""Host channel of the stage sessions (`zkp_channel_*`, include/zkp.h): winter-prover's
ProverChannel over DefaultRandomCoin<Blake3_256>. Host-only (no device): replayed
against the CPU oracle's own transcript for the same proof — every draw (composition
coefficients, z, DEEP coefficients, FRI alphas), the grinding seed's nonce check and
the query positions must come out identical."""
import pytest

import oracle_ref as O
from proof_format import sections
from zk_stark_project_amd import AIR_GLOBAL_UPDATE, AIR_MIMC, MimcProver, ProofOptions, _native
from zk_stark_project_amd.field import to_bytes


def felts(b: bytes):
    return [int.from_bytes(b[i:i + 16], "little") for i in range(0, len(b), 16)]


def replay(air_id, data: bytes, w, n, pub, opts, ce, C):
    proof, st = O.prove_stages(air_id, data, w, n, to_bytes(pub), opts, ce, C)
    sec = sections(proof)
    com = sec["commitments"]
    L = len(felts(st["alphas"]))
    ch = _native.Channel(air_id, w, n, pub, opts)
    try:
        ch.commit(com[0:32])
        assert ch.draw_coeffs(opts.batching_constraints, len(felts(st["coeffs"]))) == felts(st["coeffs"])
        ch.commit(com[32:64])
        z = ch.draw()
        ood = felts(st["ood"])
        ch.commit_felts(ood[:2 * w])
        ch.commit_felts(ood[2 * w:])
        assert ch.draw_coeffs(opts.batching_deep, w + C) == felts(st["deep_coeffs"])
        alphas = []
        for layer in range(L):
            ch.commit(com[64 + 32 * layer:96 + 32 * layer])
            alphas.append(ch.draw())
        assert alphas == felts(st["alphas"])
        ch.commit(com[-32:])
        seed = ch.seed()
        nonce = sec["nonce"]
        if opts.grinding_factor:  # the nonce meets the grinding bits on this seed
            h = O.blake3(seed + nonce.to_bytes(8, "little"))
            v = int.from_bytes(h[:8], "little")
            assert v & ((1 << opts.grinding_factor) - 1) == 0
        pos = ch.query_positions(nonce)
        assert len(pos) == len(set(pos)) and pos == sorted(pos)
        return z, pos, proof
    finally:
        ch.close()


@pytest.mark.parametrize("n,blowup,grind", [(64, 8, 4), (256, 16, 8)])
def test_channel_replays_oracle_mimc(n, blowup, grind):
    opts = ProofOptions(40, blowup, grind)
    p = MimcProver(opts)
    trace = p.build_trace(42 * 10**6, n)
    pub = p.get_pub_inputs(trace).to_elements()
    _, otr = O.prove(AIR_MIMC, trace.to_bytes(), 1, n, to_bytes(pub), opts)
    z, pos, _ = replay(AIR_MIMC, trace.to_bytes(), 1, n, pub, opts, 8, 6)
    assert z == int(otr.z.lo) | (int(otr.z.hi) << 64)
    assert pos == [int(otr.query_positions[i]) for i in range(otr.num_unique_queries)]


def test_channel_replays_oracle_global_update():
    from test_gpu_parity import gu_prover
    opts = ProofOptions(40, 16, 4)
    p = gu_prover(6, 64, opts, seed=6)
    trace = p.build_trace()
    pub = p.get_pub_inputs(trace).to_elements()
    _, otr = O.prove(AIR_GLOBAL_UPDATE, trace.to_bytes(), 120, 64, to_bytes(pub), opts)
    z, pos, _ = replay(AIR_GLOBAL_UPDATE, trace.to_bytes(), 120, 64, pub, opts, 2, 1)
    assert z == int(otr.z.lo) | (int(otr.z.hi) << 64)
    assert pos == [int(otr.query_positions[i]) for i in range(otr.num_unique_queries)]


def test_channel_arguments():
    opts = ProofOptions(40, 8, 4)
    with pytest.raises(_native.ZkpError) as e:
        _native.Channel(AIR_MIMC, 1, 100, [0, 0], opts)  # n not a power of two
    assert e.value.code == 3
    ch = _native.Channel(AIR_MIMC, 1, 64, [1, 2], opts)
    with pytest.raises(_native.ZkpError):
        ch.draw_coeffs(7, 3)  # no such batching method
    ch.close()
