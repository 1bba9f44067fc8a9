#!/bin/bash
# GPU suite, smoke and the bench lines of c2 (default), c3, c4, c5; then optional variant A/B
# (tools/var_phases.sh) on the listed workloads.  Output: gpurun_out/$1
# usage: tools/gpu_bench_lines.sh NAME ["variants" "workloads"]
set -e
O=gpurun_out/${1:-bench_lines}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --cpu-budget 6 > $O/bench_$w.log 2>&1
done
if [ -n "$2" ]; then
  for w in ${3:-c3}; do bash tools/var_phases.sh ${1:-bench_lines}/$w "$2" $w; done
fi
echo bench_lines_done
