set -e
O=gpurun_out/r05_b11; mkdir -p $O
export TMPDIR=/tmp
MPCB_LIB=mpc_blaster_amd/variants/lib_asord.so timeout -k 10 300 python tools/ab_as_order.py 20 > $O/ab_as_order.txt 2>&1
echo b9_done
