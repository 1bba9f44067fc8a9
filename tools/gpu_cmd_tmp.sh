set -e
O=gpurun_out/r05_b3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --workload c4 --cpu-budget 4 > $O/bench_c4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c4 -o run -- python3 bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --no-latency > $O/stats_c4.log 2>&1
MPCB_LIB=mpc_blaster_amd/variants/lib_stamps.so timeout -k 10 120 python tools/wave_times_p2.py c3 8 > $O/wave_times_p2_c3.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.log 2>&1
echo b3_done
