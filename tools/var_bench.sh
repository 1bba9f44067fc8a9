#!/bin/bash
# usage: scratch/var_bench.sh "name1 name2 ..." [bench args]
export TMPDIR=/tmp
V=$1; shift
for v in base $V; do
  if [ "$v" = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/var_$v.log 2>&1 || { echo "fail $v"; exit 1; }
done
