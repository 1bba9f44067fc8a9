set -e
O=gpurun_out/r05_b19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q -s --timeout 150 --timeout-method thread -k "17 or 20 or 24 or 27 or 28 or 10 or 30" > $O/fuzz.log 2>&1 || true
echo b19_done
