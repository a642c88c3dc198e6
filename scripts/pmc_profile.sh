#!/bin/bash
# Collect rocprofv3 PMC counters for bench.py, one counter group per pass
# (gfx950 pass limits; never combined with --sys-trace etc.). Output: gpurun_out/pmc/<tag>/...
set -u
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $ROOT/bench.py $ARGS > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
