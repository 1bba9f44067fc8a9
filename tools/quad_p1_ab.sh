#!/bin/bash
# A/B of the quad-lane rollout (MPCB_QUAD_P1_MAX) at the large-chunk workloads c3, c5, c4.
# Output: gpurun_out/r03_s2_quad
set -e
O=gpurun_out/r03_s2_quad; mkdir -p $O
export TMPDIR=/tmp
for rep in a b; do
for w in c3 c5 c4; do
  for v in def quad; do
    if [ $v = quad ]; then export MPCB_QUAD_P1_MAX=1048576; else unset MPCB_QUAD_P1_MAX; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload $w --steps 30 --warmup 10 > $O/${w}${rep}_$v.log 2>&1
    python3 -c "import json; d=json.loads(open('$O/${w}${rep}_$v.log').read().strip().splitlines()[-1]); print('$w $rep $v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['roofline']['phase_ms'].items()})"
  done
done
done
