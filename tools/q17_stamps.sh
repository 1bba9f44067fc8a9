#!/bin/bash
# Per-region cycle stamps of the 16-lane 17/6 kernel (diagnostic build, workgroup 0):
#   python tools/build_variant.py q17st -DMPCB_Q17_STAMPS=1   (here), then on the GPU box:
#   bash tools/q17_stamps.sh [bench_full17 args]
# Prints the interior point's phase totals (ipm) and the first backward / forward pass (bwd, fwd).
MPCB_LIB=mpc_blaster_amd/variants/lib_q17st.so timeout -k 10 120 python tools/bench_full17.py --steps 1 --warmup 0 "$@" > /tmp/q17st.log 2>&1
grep -m 2 "QSTAMP ipm" /tmp/q17st.log; grep -m 1 "QSTAMP bwd" /tmp/q17st.log; grep -m 1 "QSTAMP fwd" /tmp/q17st.log; grep -c "QSTAMP bwd" /tmp/q17st.log
