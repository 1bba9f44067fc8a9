#!/bin/bash
# Round-end validation on the GPU box: full GPU suite, smoke, default bench, the bench through
# torch.distributed.run (1 rank: the multi-GPU code path) and through its own launcher, profiles
# (tools/collect_profiles.sh: rocprofv3 kernel stats + PMC for c2..c5), the 17/6 benches with
# kernel stats and PMC of the unconstrained and boxed interior-point kernels, and the batched
# 17/6 closed loop.  Output: gpurun_out/$1.  PART=1: everything up to the c2..c5 profiles;
# PART=2: the 17/6 part (two calls that each fit gpurun's limit); default both.
set -e
O=gpurun_out/${1:-round_end}; mkdir -p $O
export TMPDIR=/tmp
PART=${PART:-all}
if [ "$PART" != 2 ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_torchrun.log 2>&1
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --cpu-budget 6 > $O/bench_$w.log 2>&1
done
bash tools/collect_profiles.sh ${1:-round_end}
fi
if [ "$PART" != 1 ]; then
for b in none input all; do
  timeout -k 10 200 python tools/bench_full17.py --bounds $b --steps 5 > $O/bench_full17_$b.log 2>&1
done
timeout -k 10 200 python tools/bench_full17.py --dtype f32 --batch 16384 --steps 5 > $O/bench_full17_f32.log 2>&1
timeout -k 10 200 python tools/bench_loop17.py > $O/bench_loop17.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_full17 -o run -- \
  python3 tools/bench_full17.py --steps 5 > $O/stats_full17.log 2>&1
PROG=tools/bench_full17.py bash tools/profile_pmc.sh $O/pmc_full17 --bounds none --steps 2 --warmup 1
python3 tools/pmc_summary.py $O/pmc_full17 --json $O/pmc_full17.json > $O/pmc_full17.txt
bash tools/profile_full17_box.sh ${1:-round_end}
fi
echo round_end_done
