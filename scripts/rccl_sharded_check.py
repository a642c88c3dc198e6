"""RCCL backend check of the coset-sharded prover.

Run one process per rank:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 scripts/rccl_sharded_check.py [--same-device] [--log-n 12]
Every rank proves the same MiMC trace through its RCCL communicator; rank 0
compares the bytes with a single-GPU proof. `--same-device` puts all ranks on
GPU 0 (a one-GPU box; RCCL may refuse duplicate devices, which is reported).
Exit status 0 = identical proofs on every rank.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--log-n", type=int, default=12)
    args = ap.parse_args()
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from zk_stark_project_amd import AIR_MIMC, MimcProver, ProofOptions, _native
    from zk_stark_project_amd.sharded import rccl_group_comm
    dev = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    ctx = _native.Context(dev)
    opts = ProofOptions(40, 8, 12)
    p = MimcProver(opts, ctx)
    trace = p.build_trace(42 * 10**6, 1 << args.log_n)
    pub = p.get_pub_inputs(trace).to_elements()
    comm = rccl_group_comm(ctx, rank, world)
    data, _ = ctx.prove_sharded(comm, AIR_MIMC, trace.data, pub, opts)
    ok = True
    if rank == 0:
        ref, _ = ctx.prove(AIR_MIMC, trace.data, pub, opts)
        ok = data == ref
    import torch
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(f"RCCL sharded proof over {world} ranks identical to single-GPU proof: {bool(flag.item())}")
    comm.close()
    dist.destroy_process_group()
    sys.exit(0 if flag.item() else 1)


if __name__ == "__main__":
    main()
