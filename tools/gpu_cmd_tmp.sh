set -e
O=gpurun_out/r05_b8; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_c2.sh $O main nohand
for ch in 65536 131072; do MPCB_CHUNK=$ch timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline > $O/c5_chunk$ch.log 2>&1; done
echo b8_done
