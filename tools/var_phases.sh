#!/bin/bash
# Per-phase device times (bench.py roofline.phase_ms) of library variants on one workload, twice.
# usage: tools/var_phases.sh OUTDIR "variant names" [workload]
set -e
O=gpurun_out/$1; mkdir -p $O; V=$2; W=${3:-c2}
export TMPDIR=/tmp
for rep in a b; do
  for v in base $V; do
    if [ $v = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload $W --steps 50 --warmup 20 > $O/${W}${rep}_$v.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/${W}${rep}_$v.log').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['roofline']['phase_ms'].items()})"
  done
done
