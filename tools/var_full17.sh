#!/bin/bash
# A/B of library variants on the 17/6 benches (none / input / all), twice each.
# usage: tools/var_full17.sh OUTDIR "variant names"
set -e
O=gpurun_out/$1; mkdir -p $O; V=$2
export TMPDIR=/tmp
for rep in a b; do
  for v in base $V; do
    if [ $v = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
    for b in none input all; do
      timeout -k 10 200 python tools/bench_full17.py --bounds $b --steps 5 > $O/${b}${rep}_$v.log 2>&1
      python3 -c "import json; d=json.loads(open('$O/${b}${rep}_$v.log').read().strip().splitlines()[-1]); print('$rep $v $b', round(d['phase_ms']['riccati'],3), d['status_counts'])"
    done
  done
done
