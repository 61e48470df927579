#!/bin/bash
# Copies the results of scripts/gpu_r05_final.sh (gpurun_out/final5, gpurun_out/pmc) into the tracked profiles/
# under round-5 names: bench lines, PMC summaries (json + text), kernel trace statistics per workload, the
# two-process record, the host probe and the GPU test summary.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
F=$R/gpurun_out/final5
P=$R/profiles
for w in c2 c3 c4 c5 c6; do
  grep '^{' "$F/bench_$w.log" | tail -n 1 > "$P/r05_${w}_bench.json"
done
for w in c2 c3 c4 c6; do
  cp "$R/gpurun_out/pmc/pmc_$w.json" "$P/pmc_$w.json"
  cp "$R/gpurun_out/pmc/$w/summary.txt" "$P/r05_pmc_${w}_summary.txt"
done
for w in c2 c3 c4 c5 c6; do
  cp "$F/prof_$w/run_kernel_stats.csv" "$P/r05_${w}_rocprof_kernel_stats.csv"
done
grep '^{' "$F/two_proc.log" > "$P/r05_shard_two_proc.json.txt" || true
cp "$F/host_probe.log" "$P/r05_shard_host_probe.txt"
tail -n 3 "$F/pytest_gpu.log" > "$P/r05_gpu_tests.txt"
echo collected
