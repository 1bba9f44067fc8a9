set -e
O=gpurun_out/r05_b24; mkdir -p $O
export TMPDIR=/tmp
for v in tol17 tol17b; do
  MPCB_LIB=mpc_blaster_amd/variants/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz17.py tests/test_gpu_full17.py -q -s --timeout 200 --timeout-method thread -k "fp32 or 1 or 5 or 8 or 9 or 13" > $O/fuzz17_$v.log 2>&1 || true
done
echo b24_done
