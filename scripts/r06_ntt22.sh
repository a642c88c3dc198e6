#!/bin/bash
# 2^21-2^22 pass plans at the C4-rank shape (tests/native/kbench_ntt 22 rank), tuning only.
set -o pipefail
mkdir -p gpurun_out
for v in kbench_ntt kbench_ntt_p1210 kbench_ntt_p1111 kbench_ntt kbench_ntt_p1210 kbench_ntt_p1111; do
  echo "== $v"
  timeout -k 10 90 ./tests/native/$v 22 rank || exit 1
done > gpurun_out/kbench_ntt22_plans.txt 2>&1
cat gpurun_out/kbench_ntt22_plans.txt
