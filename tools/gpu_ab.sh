#!/bin/bash
# A/B on the GPU box: full GPU suite and smoke on the in-tree library, then per-phase times of the
# in-tree library against variant libraries (tools/build_variant.py) on each workload.
# usage: tools/gpu_ab.sh NAME "variants" "workloads"   Output: gpurun_out/NAME
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for w in ${3:-c2}; do
  bash tools/var_phases.sh ${1:-ab}/$w "$2" $w
done
echo ab_done
