#!/bin/bash
# A/B on the GPU box: GPU tests against each variant (MPCB_LIB), then c2 (twice), c3, c4 benches.
# usage: tools/ab_run.sh OUTDIR "variant names" [workloads, default "c2 c3"]
set -e
O=gpurun_out/$1; mkdir -p $O; V=$2; WL=${3:-c2 c3}
export TMPDIR=/tmp
for v in $V; do
  export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_parity.py::test_library_is_the_native_hip_build > $O/tests_$v.log 2>&1
done
for rep in a b; do
  for v in base $V; do
    if [ $v = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
    for w in $WL; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload $w > $O/${w}${rep}_$v.log 2>&1
    done
  done
done
echo ab_done
