#!/bin/bash
# 17/6 benches (none / input / all) twice, one JSON summary line each.  usage: tools/full17_quick.sh OUTDIR
set -e
O=gpurun_out/${1:-full17q}; mkdir -p $O
export TMPDIR=/tmp
for rep in a b; do
  for b in none input all; do
    timeout -k 10 200 python tools/bench_full17.py --bounds $b --steps 5 > $O/${b}_$rep.log 2>&1
    python3 -c "import json; d=json.loads(open('$O/${b}_$rep.log').read().strip().splitlines()[-1]); print('$rep $b', round(d['ms_per_step'],3), d['status_counts'], {k: round(v,3) for k,v in d['phase_ms'].items()})"
  done
done
