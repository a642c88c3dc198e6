#!/bin/bash
# NTT pass plans at the TrainingUpdate shape (2^13, 64 columns x 16 cosets), tuning only.
set -o pipefail
mkdir -p gpurun_out
for v in kbench_ntt kbench_ntt_k5 kbench_ntt_k7 kbench_ntt_k8 kbench_ntt_1p; do
  echo "== $v"
  timeout -k 10 60 ./tests/native/$v 13 tu || exit 1
done > gpurun_out/kbench_ntt13.txt 2>&1
cat gpurun_out/kbench_ntt13.txt
timeout -k 10 120 ./tests/native/kbench_ntt 20 > gpurun_out/kbench_ntt20_pipe.txt 2>&1 || { tail -5 gpurun_out/kbench_ntt20_pipe.txt; exit 1; }
cat gpurun_out/kbench_ntt20_pipe.txt
