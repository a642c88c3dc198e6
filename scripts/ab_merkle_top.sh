#!/bin/bash
# A/B of the Merkle upper-level schedule (ZKP_MERKLE_LANE_MIN = log2 of the node
# count down to which lane passes run before the LDS-fused top), C2 device-resident.
set -o pipefail
for k in 18 14 12 10; do
  ZKP_MERKLE_LANE_MIN=$k timeout -k 10 120 python3 bench.py --steps 30 --no-cpu-baseline --no-verify --sustain-s 0 \
    > gpurun_out/ab_mt_$k.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_mt_$k.json').read().strip().splitlines()[-1]); print('lane_min=$k', d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'])"
done
