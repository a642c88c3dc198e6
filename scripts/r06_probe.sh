#!/bin/bash
# Round-6 probes (GPU box): cold-start breakdown of C3, the NTT kernel bench at the C2
# and C4-rank shapes, each step time-limited, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python3 scripts/first_proof_probe.py --air agg > gpurun_out/fpp_agg.json 2> gpurun_out/fpp_agg.err || { tail -5 gpurun_out/fpp_agg.err; exit 1; }
timeout -k 10 120 ./tests/native/kbench_ntt 20 > gpurun_out/kbench_ntt20.txt 2>&1 || { tail -5 gpurun_out/kbench_ntt20.txt; exit 1; }
timeout -k 10 120 ./tests/native/kbench_ntt 22 rank > gpurun_out/kbench_ntt22.txt 2>&1 || { tail -5 gpurun_out/kbench_ntt22.txt; exit 1; }
cat gpurun_out/kbench_ntt20.txt gpurun_out/kbench_ntt22.txt
echo PROBEOK
