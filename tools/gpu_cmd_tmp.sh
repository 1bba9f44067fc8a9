set -e
export TMPDIR=/tmp
O=gpurun_out/p2b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in a b; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload c2 --steps 50 --warmup 20 > $O/c2$r.log 2>&1
python3 -c "import json,sys; d=json.loads(open('$O/c2$r.log').read().strip().splitlines()[-1]); print('$r', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['roofline']['phase_ms'].items()})"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 -- python bench.py --no-cpu-baseline --no-secondary --no-latency --workload c2 --steps 50 --warmup 20 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -3
cat $(find $O/prof -name "*kernel_stats.csv" | head -1) | cut -d, -f1-8 | head -12
bash tools/env_ab.sh c4chunk c4 "ch64k=MPCB_CHUNK=65536;ch16k=MPCB_CHUNK=16384;ch8k=MPCB_CHUNK=8192"
