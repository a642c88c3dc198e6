#!/bin/bash
# Round-end measurement: C2 and C3 bench lines (C2 with the CPU baseline and the oracle
# check), the C2 timeline, then rocprofv3 kernel-trace + PMC passes for C2 and C3.
#   scripts/round_end.sh <tag>   -> gpurun_out/b_c2.json, b_c3.json, timeline_<tag>.txt, prof_<tag>{,agg}/
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --stats > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
timeout -k 10 240 python bench.py --air agg --steps 10 --no-cpu-baseline --stats > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || { tail -20 gpurun_out/b_c3.err; exit 1; }
timeout -k 10 120 python3 scripts/timeline.py > gpurun_out/timeline_$TAG.txt 2>&1 || { tail -5 gpurun_out/timeline_$TAG.txt; exit 1; }
bash scripts/profile_round.sh $TAG || exit 1
bash scripts/profile_round.sh ${TAG}agg --air agg || exit 1
python3 -c "
import json
for f in ['b_c2','b_c3']:
    d=json.loads(open('gpurun_out/'+f+'.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['launches']['per_proof'])
"
