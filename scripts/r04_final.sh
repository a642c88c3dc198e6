#!/bin/bash
# Round-4 closing run on one box: the full GPU suite, smoke(), the C2 headline line (default
# steps, CPU baseline), the C3 line, the C2 timeline, and the rocprofv3 kernel-trace + PMC
# passes for C2 and C3 (scripts/profile_round.sh). Every step under its own time limit.
set -o pipefail
TAG=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu --durations=10 \
  > gpurun_out/final_suite.log 2>&1 || { tail -40 gpurun_out/final_suite.log; exit 1; }
tail -3 gpurun_out/final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_c2.json 2> gpurun_out/final_c2.err || { tail -20 gpurun_out/final_c2.err; exit 1; }
timeout -k 10 300 python bench.py --air agg --steps 20 --no-cpu-baseline > gpurun_out/final_c3.json 2> gpurun_out/final_c3.err || { tail -20 gpurun_out/final_c3.err; exit 1; }
python3 -c "
import json
for f in ['final_c2','final_c3']:
    d=json.loads(open('gpurun_out/'+f+'.json').read().strip().splitlines()[-1])
    r=d['roofline']
    print(f, d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], r['frac'], r['avg_launch_ms'], r.get('valu_floor_frac'), d['session']['session_ms'], (d.get('cpu_baseline') or {}).get('value'))
"
timeout -k 10 120 python3 scripts/timeline.py > gpurun_out/timeline_$TAG.txt 2>&1 || { tail -5 gpurun_out/timeline_$TAG.txt; exit 1; }
bash scripts/profile_round.sh $TAG || exit 1
bash scripts/profile_round.sh ${TAG}agg --air agg || exit 1
echo final-done
