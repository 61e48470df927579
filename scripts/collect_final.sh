#!/bin/bash
# Copies the results of scripts/gpu_r03_final.sh (gpurun_out/final, gpurun_out/pmc) into the tracked profiles/
# under round-3 names: bench lines, PMC summaries (json + text), the C2 kernel trace statistics, the shard
# probe and the two-process record.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
F=$R/gpurun_out/final
P=$R/profiles
for w in c2 c3 c4 c5 c6; do
  tail -n 1 "$F/bench_$w.log" > "$P/r03_${w}_bench.json"
done
for w in c2 c3 c4 c6; do
  cp "$R/gpurun_out/pmc/pmc_$w.json" "$P/pmc_$w.json"
  cp "$R/gpurun_out/pmc/$w/summary.txt" "$P/r03_pmc_${w}_summary.txt"
done
cp "$F/prof_c2/run_kernel_stats.csv" "$P/r03_c2_rocprof_kernel_stats.csv"
cp "$F/prof_probe/probe_kernel_stats.csv" "$P/r03_shard_probe_kernel_stats.csv"
grep "^{" "$F/probe.log" | tail -n 1 > "$P/r03_shard_probe.json"
grep '^{' "$F/two_proc.log" > "$P/r03_shard_two_proc.json.txt"
tail -n 3 "$F/pytest_gpu.log" > "$P/r03_gpu_tests.txt"
echo collected
