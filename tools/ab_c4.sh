#!/bin/bash
# c4 A/B of library variants (tools/build_variant.py), interleaved: one bench line per variant and
# repetition.  usage (GPU box): bash tools/ab_c4.sh OUTDIR VARIANT... (main = the in-tree library)
set -e
O=$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then L=mpc_blaster_amd/libmpcblaster.so; else L=mpc_blaster_amd/variants/lib_$v.so; fi
    MPCB_LIB=$L timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --steps 20 --warmup 3 > $O/c4_${v}_$rep.log 2>&1
    tail -1 $O/c4_${v}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$v rep $rep: %.4f ms/step, active-set %.4f ms, P2 %.4f ms' % (d['ms_per_step'], r['phase_ms']['forward'], r['phase_ms']['riccati']))" | tee -a $O/summary.txt
  done
done
