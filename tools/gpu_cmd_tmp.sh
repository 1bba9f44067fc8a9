set -e
O=gpurun_out/r05_b14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -v -s --timeout 120 --timeout-method thread -k order > $O/edges.log 2>&1
echo b14_done
