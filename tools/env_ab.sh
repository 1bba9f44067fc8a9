#!/bin/bash
# Per-phase device times of the in-tree library under environment overrides, alternating twice.
# usage: tools/env_ab.sh OUTDIR WORKLOAD "NAME=ENV1 ENV2;NAME2=ENV3" [pytest -k expr]
# e.g.   tools/env_ab.sh fuse c2 "two=MPCB_FUSE_P12=0;one=" "c2 or iterate"
set -e
O=gpurun_out/$1; mkdir -p $O; W=$2; CASES=$3; K=${4:-}
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
IFS=';' read -ra CS <<< "$CASES"
for rep in a b; do
  for c in "${CS[@]}"; do
    name=${c%%=*}; envs=${c#*=}
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload $W --steps 50 --warmup 20 > $O/${W}${rep}_$name.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/${W}${rep}_$name.log').read().strip().splitlines()[-1]); print('$rep $name', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['roofline']['phase_ms'].items()})"
  done
done
