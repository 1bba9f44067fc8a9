#!/bin/bash
# 17/6 boxed runs on the GPU box: the bench lines, rocprofv3 kernel stats and the PMC passes of the
# interior-point kernels riccati17q_kernel<double, true, true> (input box, Mehrotra) and
# <double, true, false> (input + state box, with the polish).  Output: gpurun_out/$1
set -e
O=gpurun_out/${1:-full17_box}; mkdir -p $O
export TMPDIR=/tmp
for b in input all; do
  timeout -k 10 200 python tools/bench_full17.py --bounds $b --steps 5 > $O/bench_full17_$b.log 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_full17_$b -o run -- \
    python3 tools/bench_full17.py --bounds $b --steps 3 > $O/stats_full17_$b.log 2>&1
  PROG=tools/bench_full17.py bash tools/profile_pmc.sh $O/pmc_full17_$b --bounds $b --steps 1 --warmup 1
  python3 tools/pmc_summary.py $O/pmc_full17_$b --json $O/pmc_full17_$b.json > $O/pmc_full17_$b.txt
done
echo full17_box_done
