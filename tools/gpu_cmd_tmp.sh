set -e
export TMPDIR=/tmp
O=gpurun_out/p1stg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "c2 or iterate or c1 or linearize or small or closed_loop" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in a b; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-latency --workload c2 --steps 50 --warmup 20 > $O/c2$r.log 2>&1
python3 -c "import json,sys; d=json.loads(open('$O/c2$r.log').read().strip().splitlines()[-1]); print('$r', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['roofline']['phase_ms'].items()})"
done
