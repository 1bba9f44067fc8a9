set -e
O=gpurun_out/r05_b27; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q -s --timeout 150 --timeout-method thread > $O/fuzz.log 2>&1 || true
echo b27_done
