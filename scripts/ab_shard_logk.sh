#!/bin/bash
# One-rank device work (world 8) with the leaf-digest all-to-all in 1, 2, 4 chunks.
set -o pipefail
mkdir -p gpurun_out
for air in agg mimc; do
  for k in 0 1 2; do
    ZKP_SHARD_LOGK=$k timeout -k 10 240 python -u scripts/rank_emulate.py --air $air --world 8 --rank 0 > gpurun_out/emu_k.log 2>&1 \
      || { tail -20 gpurun_out/emu_k.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/rank_emulate_${air}_w8_r0.json')); k=d['kernels']; print('$air logK=$k', d['kernel_ms_per_proof'], 'leaf_hash_shard', k.get('leaf_hash_shard'))"
  done
done
