#!/bin/bash
# P1 A/B on the GPU box: full GPU suite and smoke on the in-tree library, then per-phase times of
# the in-tree library against variant libraries (tools/build_variant.py); with a third argument
# also the default bench line and the c2 profiles.  Output: gpurun_out/$1
set -e
O=gpurun_out/${1:-p1ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/var_phases.sh ${1:-p1ab}/c2 "${2:-noown}" c2
if [ -n "$3" ]; then   # then the c2 bench line and its profiles
  timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
  WORKLOADS=c2 bash tools/collect_profiles.sh ${1:-p1ab}
fi
echo p1ab_done
