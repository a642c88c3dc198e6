#!/bin/bash
# GPU: DEEP occupancy variant (parity subset + C2 A/B) and the one-rank emulations on the final code.
set -o pipefail
mkdir -p gpurun_out
ZKP_LIB=build_exp/deep/x/libzkp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_parity.py > gpurun_out/deep_tests.log 2>&1 || { tail -30 gpurun_out/deep_tests.log; exit 1; }
tail -1 gpurun_out/deep_tests.log
bash scripts/ab_libs.sh zk_stark_project_amd/libzkp.so build_exp/deep/x/libzkp.so > gpurun_out/ab_deep.txt 2>&1 || { tail -5 gpurun_out/ab_deep.txt; exit 1; }
cat gpurun_out/ab_deep.txt
bash scripts/rank_emulate.sh || exit 1
