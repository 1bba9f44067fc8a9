set -e
O=gpurun_out/p2dpp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/env_ab.sh p2dpp c2 "notan=MPCB_P1_TAN=0;tan=MPCB_P1_TAN=1"
MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_stamps.so MPCB_P1_TAN=1 timeout -k 10 120 python tools/stamps.py c2 > $O/stamps_tan.txt 2>&1
head -14 $O/stamps_tan.txt
