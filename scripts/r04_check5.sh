#!/bin/bash
# GPU check: the GlobalUpdate / stage tests on the coalesced lazy-GU leaf build
# (build_exp/gu), a C3 A/B against the committed library, and a C2 line with the
# concurrent leg.
set -o pipefail
mkdir -p gpurun_out
ZKP_LIB=build_exp/gu/x/libzkp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  -k "global or agg or gu or stages or sharded or trace" > gpurun_out/gu_tests.log 2>&1 || { tail -40 gpurun_out/gu_tests.log; exit 1; }
tail -2 gpurun_out/gu_tests.log
bash scripts/ab_libs.sh zk_stark_project_amd/libzkp.so build_exp/gu/x/libzkp.so --air agg --steps 10 > gpurun_out/ab_gu.txt 2>&1 || { tail -5 gpurun_out/ab_gu.txt; exit 1; }
cat gpurun_out/ab_gu.txt
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/b_c2c.json 2> gpurun_out/b_c2c.err || { tail -20 gpurun_out/b_c2c.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b_c2c.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['concurrent'])
"
