#!/bin/bash
# Kernel-level view of the sharded proof's per-rank work on one GPU: the new
# comm tests, then rocprofv3 kernel traces of the in-process group at world 1
# and world 8 for C4 (MiMC 2^22) and C5 (GlobalUpdate 2^20 x 120).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py \
  > gpurun_out/comm_tests.log 2>&1 || { tail -30 gpurun_out/comm_tests.log; exit 1; }
tail -2 gpurun_out/comm_tests.log
for air in mimc agg; do
  for w in 1 8; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sh_${air}_w$w -o run -- \
      python3 scripts/sharded_rank_work.py --air $air --worlds $w --steps 2 > gpurun_out/prof_sh_${air}_w$w.log 2>&1 \
      || { tail -20 gpurun_out/prof_sh_${air}_w$w.log; exit 1; }
    grep world gpurun_out/prof_sh_${air}_w$w.log
  done
done
echo PROFOK
