set -e
O=gpurun_out/r05_b25; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py -v -s --timeout 150 --timeout-method thread > $O/edges.log 2>&1 || true
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q -s --timeout 150 --timeout-method thread > $O/fuzz.log 2>&1 || true
timeout -k 10 400 python tools/box_ipm_direct.py > $O/box_ipm_direct.txt 2>&1 || true
bash tools/ab_c4.sh $O main prefb
echo b25_done
