#!/bin/bash
# A/B of the active-set kernel at 3 waves per SIMD (MPCB_AS_WAVES=3 build under
# mpc_blaster_amd/variants/lib_w3.so): rocprofv3 kernel stats of the c4 bench per library, twice.
set -e
O=gpurun_out/${1:-r06/ring}; mkdir -p $O
export TMPDIR=/tmp
for rep in a b; do
  for v in base w3; do
    lib=$PWD/mpc_blaster_amd/libmpcblaster.so
    [ $v != base ] && lib=$PWD/mpc_blaster_amd/variants/lib_$v.so
    MPCB_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v$rep -o run -- \
      python3 bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-latency > $O/$v$rep.log 2>&1
    python3 -c "
import csv
for r in csv.DictReader(open('$O/$v$rep/run_kernel_stats.csv')):
    if 'as_' in r['Name'] or 'riccati' in r['Name']: print('$rep $v', r['Name'].split('(')[0][-40:], round(float(r['AverageNs'])/1e3, 1))
"
  done
done
