#!/bin/bash
# GPU check: the non-slow GPU suite, a C2 line with the per-kernel table, the FRI-tail
# phase probe (instrumented build) and the concurrency probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m "gpu and not slow" \
  > gpurun_out/check_tests.log 2>&1 || { tail -40 gpurun_out/check_tests.log; exit 1; }
tail -2 gpurun_out/check_tests.log
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --stats > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b_c2.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step'], d['pcie_inclusive']['ms_per_proof'], d['sustained']['proofs_per_s'])
"
grep -E "fri_fold16|fri_tail|merkle_fri" gpurun_out/b_c2.err
ZKP_LIB=build_exp/ts/x/libzkp.so timeout -k 10 120 python scripts/tail_ts.py > gpurun_out/tail_ts.txt 2>&1 || { tail -5 gpurun_out/tail_ts.txt; exit 1; }
timeout -k 10 200 python scripts/concurrency_probe.py mimc 2 > gpurun_out/conc.txt 2>&1 || { tail -5 gpurun_out/conc.txt; exit 1; }
cat gpurun_out/tail_ts.txt gpurun_out/conc.txt
bash scripts/ab_libs.sh build_exp/base/x/libzkp.so zk_stark_project_amd/libzkp.so > gpurun_out/ab_quad.txt 2>&1 || { tail -5 gpurun_out/ab_quad.txt; exit 1; }
cat gpurun_out/ab_quad.txt
