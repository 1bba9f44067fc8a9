#!/bin/bash
# Round-6 end runs on the GPU box, in parts that each fit one gpurun call (tools/round_end.sh's
# steps).  PART=bench: default bench, torch.distributed.run, c3-c5 lines, c2 at 2x / 4x the batch
# (waves per SIMD); PART=prof: WORKLOADS=... tools/collect_profiles.sh; PART=17: the
# 17/6 part of tools/round_end.sh.  Output: gpurun_out/$1.
set -e
O=gpurun_out/${1:-r06_end}; mkdir -p $O
export TMPDIR=/tmp
case "$PART" in
bench)
  timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_torchrun.log 2>&1
  for w in c3 c4 c5; do
    timeout -k 10 300 python bench.py --workload $w --cpu-budget 6 > $O/bench_$w.log 2>&1
  done
  for b in 8192 16384; do
    timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-secondary --no-latency --steps 50 --warmup 10 > $O/bench_c2_b$b.log 2>&1
  done
  ;;
prof)
  bash tools/collect_profiles.sh ${1:-r06_end}
  ;;
17)
  PART=2 bash tools/round_end.sh ${1:-r06_end}
  ;;
esac
echo part_done
