#!/bin/bash
# A/B of the row-major export records padded to whole cache lines (MPCB_REC_PAD=1 build under
# mpc_blaster_amd/variants/lib_pad.so): c4 box parity tests on the variant, rocprofv3 kernel stats
# of the c4 bench per library (twice), and the as_kernel's FETCH_SIZE / WRITE_SIZE per library.
set -e
O=gpurun_out/${1:-r06/pad}; mkdir -p $O
export TMPDIR=/tmp
MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_pad.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "c4 or box or order" > $O/tests_pad.log 2>&1
tail -1 $O/tests_pad.log
for rep in a b; do
  for v in base pad; do
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
for v in base pad; do
  lib=$PWD/mpc_blaster_amd/libmpcblaster.so
  [ $v != base ] && lib=$PWD/mpc_blaster_amd/variants/lib_$v.so
  for P in FETCH_SIZE WRITE_SIZE; do
    MPCB_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/pmc_$v -o $P -- \
      python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-latency > $O/pmc_${v}_$P.log 2>&1
  done
  python3 tools/pmc_summary.py $O/pmc_$v > $O/pmc_$v.txt 2>&1 || true
  grep -A3 -E "as_kernel_f32<true, false>|riccati_kernel_f32<true" $O/pmc_$v.txt | grep -E "as_kernel|riccati|FETCH|WRITE" | sed "s/^/$v /"
done
