#!/bin/bash
# A/B of two libzkp builds on the reference flow's proofs (tuning only):
#   scripts/ab_refflow.sh <lib A> <lib B>; alternates A and B twice; prints the warm
#   sequential 9-proof total, the TrainingUpdate proof's warm ms, device busy, and the C2 step.
set -o pipefail
A=$1; B=$2
for r in 1 2; do
  for L in "$A" "$B"; do
    out=$(ZKP_LIB=$L timeout -k 10 240 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --no-concurrent \
          --no-c3 --no-rank-emulation --no-tampered --steps 20) || exit 1
    echo "$L $(echo "$out" | python -c '
import json,sys
d=json.loads(sys.stdin.readline()); rf=d["reference_flow"]; tp=rf["training_proof_profile"]
print("warm_total", rf["warm"]["prove_ms_total"], "tu", tp["warm_ms_per_proof"], "busy", tp["device_busy_ms_per_proof"],
      "conc4", rf["warm_concurrent"][0]["prove_ms_total"], "c2", d["ms_per_step"])')"
  done
done
