#!/bin/bash
# A/B of the default library against variants/lib_<name>.so on the bench (+ c2 stamps build).
# usage: tools/ab_p2.sh OUTDIR "variant names" [bench args]
set -e
O=gpurun_out/$1; mkdir -p $O; V=$2; shift 2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
for v in base $V; do
  if [ $v = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/bench_$v.log 2>&1
done
unset MPCB_LIB
if [ -f mpc_blaster_amd/variants/lib_stamps.so ]; then
  MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_stamps.so timeout -k 10 120 python tools/stamps.py c2 > $O/stamps.log 2>&1
fi
echo done
