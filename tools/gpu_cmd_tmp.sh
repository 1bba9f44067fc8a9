set -e
O=gpurun_out/r05_b13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -v -s --timeout 120 --timeout-method thread > $O/edges.log 2>&1 || true
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/ab_c2.sh $O main prevredo
echo b13_done
