set -e
O=gpurun_out/r05_b22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/soak.py --seconds 60 > $O/soak.txt 2>&1
echo b22_done
