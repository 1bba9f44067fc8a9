#!/bin/bash
# Per-region cycle stamps of the 16-lane 17/6 kernel (diagnostic build, workgroup 0):
#   python tools/build_variant.py q17st -DMPCB_Q17_STAMPS=1   (here), then on the GPU box:
#   bash tools/q17_stamps.sh [bench_full17 args]
MPCB_LIB=mpc_blaster_amd/variants/lib_q17st.so timeout -k 10 120 python tools/bench_full17.py --steps 1 --warmup 0 "$@" | grep -v "^{" | sort | uniq -c | head -20
