#!/bin/bash
# Round profile collection on the GPU box: rocprofv3 --kernel-trace --stats of the default bench
# command, plus PMC passes (tools/profile_pmc.sh) for c2 and c3.  Output: gpurun_out/$1
set -e
OUT=gpurun_out/${1:-profiles}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_default" -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 3 > "$OUT/stats_default.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_c3" -o run -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/stats_c3.log" 2>&1
bash tools/profile_pmc.sh "$OUT/pmc_c2" --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
bash tools/profile_pmc.sh "$OUT/pmc_c3" --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/pmc_summary.py "$OUT/pmc_c2" --json "$OUT/pmc_c2.json" > "$OUT/pmc_c2.txt"
python3 tools/pmc_summary.py "$OUT/pmc_c3" --json "$OUT/pmc_c3.json" > "$OUT/pmc_c3.txt"
echo collected
