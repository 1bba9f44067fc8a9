#!/bin/bash
# Development check on the GPU box: GPU test subset (pytest -k), smoke, default bench and the c4/c5
# workloads.  Output: gpurun_out/$1.  Usage: tools/gpu_quick.sh NAME [pytest -k expr]
set -e
O=gpurun_out/${1:-quick}; mkdir -p $O
K=${2:-}
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --cpu-budget 3 > $O/bench_default.log 2>&1
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.log 2>&1
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.log 2>&1
echo quick_done
