#!/bin/bash
# merkle_top9 / merkle_upper per proof at several ZKP_MERKLE_LANE_MIN (C2, library events)
set -o pipefail
mkdir -p gpurun_out
for lm in 18 16 14 12; do
  ZKP_MERKLE_LANE_MIN=$lm timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-verify --stats > gpurun_out/lm_$lm.json 2> gpurun_out/lm_$lm.err || { tail -20 gpurun_out/lm_$lm.err; exit 1; }
  echo "lane_min=$lm $(python3 -c "import json;d=json.loads(open('gpurun_out/lm_$lm.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'])")"
  grep -E "merkle_top9|merkle_upper|fri_tail|coin " gpurun_out/lm_$lm.err
done
