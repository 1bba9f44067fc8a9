#!/usr/bin/env python3
"""Debug aid for the 16-lane 17/6 kernel: one small solve with a MPCB_Q17_DEBUG variant
(tools/build_variant.py q17dbg -DMPCB_Q17_DEBUG=1), kernel printf lines on stdout.

    MPCB_LIB=mpc_blaster_amd/variants/lib_q17dbg.so python tools/q17_debug.py [N]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_full17 import _inputs  # noqa: E402
from mpc_blaster_amd import BatchedMPC, MPCConfig  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3
x0, xref, uref, p = _inputs(1, N, 101)
m = BatchedMPC(MPCConfig.full(N=N, dtype='f64'), max_batch=1)
m.set_params(p)
m.solve(x0, xref, uref)
torch.cuda.synchronize()
print('STATUS', m.get_status().cpu().numpy().tolist())
print('U0', m.get_control().cpu().numpy().tolist())
