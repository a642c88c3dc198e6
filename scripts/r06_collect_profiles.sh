#!/bin/bash
# Copy the round-6 profile summaries from gpurun_out/ (scripts/r06_profiles.sh) into profiles/
# under the names bench.py reads (PMC_TAGS) and DESIGN.md cites. Run here, after the GPU call.
set -e
for pair in "r06_c2:mimc_c2" "r06_c3:agg_c3"; do
  tag=${pair%%:*}; wl=${pair##*:}; d=gpurun_out/prof_$tag
  cp $d/traffic.json profiles/r06_pmc_traffic_$wl.json
  cp $d/traffic.txt profiles/r06_pmc_traffic_$wl.txt
  cp $d/sq/sq.json profiles/r06_pmc_sq_$wl.json
  cp $d/sq.txt profiles/r06_pmc_sq_$wl.txt
  cp $d/trace/run_kernel_stats.csv profiles/r06_rocprof_kernel_stats_$wl.csv
done
if [ -f gpurun_out/prof_judged/run_kernel_stats.csv ]; then
  cp gpurun_out/prof_judged/run_kernel_stats.csv profiles/r06_rocprof_kernel_stats_judged.csv
  python3 scripts/judged_kernel_summary.py gpurun_out/prof_judged/run_kernel_trace.csv gpurun_out/prof_judged.json \
    > profiles/r06_judged_kernel_summary.json
  tail -1 gpurun_out/prof_judged.json > profiles/r06_bench_under_rocprof.json
fi
echo collected
