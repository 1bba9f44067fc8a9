set -e
O=gpurun_out/r05_b28; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_c4.sh $O main smaj smaj3
echo b28_done
