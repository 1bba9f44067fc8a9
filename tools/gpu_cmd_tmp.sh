set -e
O=gpurun_out/r05_b21; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/box_ipm_direct.py > $O/box_ipm_direct.txt 2>&1
echo b20_done
