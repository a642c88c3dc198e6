#!/bin/bash
# NTT exact-redo check, then a 3-way A/B: round-3 field ops (old), per-op rare
# branches (b), deferred round checks (current tree), with SQ VALU counts.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tests/native/ntt_check > gpurun_out/ntt_check.txt 2>&1 || { tail -20 gpurun_out/ntt_check.txt; exit 1; }
tail -1 gpurun_out/ntt_check.txt
for r in 1 2; do
  for L in build_exp/old/x/libzkp.so build_exp/b/x/libzkp.so zk_stark_project_amd/libzkp.so; do
    out=$(ZKP_LIB=$L timeout -k 10 180 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --steps 40) || exit 1
    echo "$L $(echo "$out" | python -c '
import json,sys
d=json.loads(sys.stdin.readline()); k=d["launches"]["by_kernel_ms"]
print(d["ms_per_step"], d["pcie_inclusive"]["ms_per_proof"], d["roofline"]["avg_launch_ms"], " ".join(f"{n}={k[n]}" for n in list(k)[:7]))')"
  done
done
bash scripts/ab_valu.sh build_exp/b/x/libzkp.so zk_stark_project_amd/libzkp.so r3
