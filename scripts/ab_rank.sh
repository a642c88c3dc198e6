#!/bin/bash
# A/B of libzkp builds on one emulated rank (tuning only):
#   scripts/ab_rank.sh <air> <world> <lib A> <lib B>
# alternates A and B twice; prints kernel ms per proof, wall ms, and the NTT launches' ms.
set -o pipefail
AIR=$1; W=$2; A=$3; B=$4
for r in 1 2; do
  for L in "$A" "$B"; do
    out=$(ZKP_LIB=$L timeout -k 10 300 python scripts/rank_emulate.py --air "$AIR" --world "$W" --steps 3 2>/dev/null) || exit 1
    echo "$L $(echo "$out" | python -c '
import json,sys
d=json.loads(sys.stdin.readline()); k=d["kernels"]
print(d["kernel_ms_per_proof"], d["wall_ms_with_host_loopback"], "ntt_dif", k["ntt_dif"], "ntt_dit", k["ntt_dit"])')"
  done
done
