#!/bin/bash
# Round profile collection on the GPU box: rocprofv3 --kernel-trace --stats of the default bench
# command and of the c3 / c4 / c5 workloads, plus PMC passes (tools/profile_pmc.sh) for each.
# Output: gpurun_out/$1 (stats_<w>/, pmc_<w>/, pmc_<w>.json|.txt)
set -e
OUT=gpurun_out/${1:-profiles}
WL=${WORKLOADS:-c2 c3 c4 c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in $WL; do
  extra="--no-cpu-baseline --no-latency"
  [ "$w" = c2 ] && extra="--cpu-budget 3 --no-latency"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_$w" -o run -- \
    python3 bench.py --workload $w --steps 20 --warmup 3 $extra > "$OUT/stats_$w.log" 2>&1
  bash tools/profile_pmc.sh "$OUT/pmc_$w" --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-latency
  python3 tools/pmc_summary.py "$OUT/pmc_$w" --json "$OUT/pmc_$w.json" > "$OUT/pmc_$w.txt"
done
echo collected
