# A/B: base vs variants on c2 (twice) and c3; stamps
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O; V=${2:-}
export TMPDIR=/tmp
for v in base $V; do
  if [ $v = base ]; then unset MPCB_LIB; else export MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_$v.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary > $O/c2a_$v.log 2>&1
  timeout -k 10 120 python bench.py --no-cpu-baseline --workload c3 > $O/c3_$v.log 2>&1
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary > $O/c2b_$v.log 2>&1
done
unset MPCB_LIB
if [ -f mpc_blaster_amd/variants/lib_stamps.so ]; then
  MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_stamps.so timeout -k 10 120 python tools/stamps.py c2 > $O/stamps.log 2>&1
fi
echo done
