set -e
export TMPDIR=/tmp
O=gpurun_out/last; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/gpu_tests.log | tail -30; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
tail -c 300 $O/bench_default.log
