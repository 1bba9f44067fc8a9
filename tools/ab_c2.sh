#!/bin/bash
# c2 A/B of library variants (tools/build_variant.py), interleaved, 3 repetitions: the default
# bench line without its secondary.  usage (GPU box): bash tools/ab_c2.sh OUTDIR VARIANT...
set -e
O=$1; shift
mkdir -p $O
for rep in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = main ]; then L=mpc_blaster_amd/libmpcblaster.so; else L=mpc_blaster_amd/variants/lib_$v.so; fi
    MPCB_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --steps 50 --warmup 5 > $O/c2_${v}_$rep.log 2>&1
    tail -1 $O/c2_${v}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$v rep $rep: %.4f ms/step, %s %.4f ms, forward %.4f ms' % (d['ms_per_step'], r['kernel'], r['kernel_ms'], r['phase_ms'].get('forward', 0)))" | tee -a $O/summary.txt
  done
done
