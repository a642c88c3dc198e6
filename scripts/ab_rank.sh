#!/bin/bash
# A/B of libzkp builds on one emulated rank (tuning only):
#   scripts/ab_rank.sh <air> <world> <lib A> <lib B>
# alternates A and B twice; prints device-busy and event-sum ms per proof, wall ms, and the NTT and tree launches' ms.
set -o pipefail
AIR=$1; W=$2; A=$3; B=$4
for r in 1 2; do
  for L in "$A" "$B"; do
    out=$(ZKP_LIB=$L timeout -k 10 300 python scripts/rank_emulate.py --air "$AIR" --world "$W" --steps 3 2>/dev/null) || exit 1
    echo "$L $(echo "$out" | python -c '
import json,sys
d=json.loads(sys.stdin.readline()); k=d["by_kernel_ms"]
print(d["device_busy_ms_per_proof"], d["kernel_event_sum_ms_per_proof"], d["wall_ms_with_host_loopback"],
      " ".join("%s=%s" % (n, k[n]) for n in ("ntt_dit", "ntt_dif", "leaf_hash_shard", "merkle_upper") if n in k))')"
  done
done
