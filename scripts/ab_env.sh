# A/B device-resident timing of one build with and without an experiment env var
# (tuning only): scripts/ab_env.sh VAR=value [bench args]; alternates 3 times.
set -e
KV=$1; shift
for r in 1 2 3 4; do
  for mode in base exp; do
    if [ $mode = exp ]; then out=$(env $KV timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --no-concurrent --steps 40 "$@")
    else out=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --no-concurrent --steps 40 "$@"); fi
    echo "$mode $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["pcie_inclusive"]["ms_per_proof"])')"
  done
done
