set -e
export TMPDIR=/tmp
O=gpurun_out/newtests; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "general_inertia or tangent_export or box or c4" > $O/gpu_tests.log 2>&1 || { grep -E "general J|PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; exit 1; }
grep -E "general J|passed|failed" $O/gpu_tests.log | tail -8
