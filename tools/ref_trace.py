"""Diagnostic (GPU box, variant library built with -DMPCB_REF_TRACE=<chunk instance>): the fp32
input box's refinement passes of that c4 instance -- per pass and input component the active sets
(lower, upper) and the refinement's verdicts (released, beyond lower, beyond upper) as stage masks.

    MPCB_LIB=mpc_blaster_amd/variants/lib_reftrace.so python tools/ref_trace.py
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = 65536, 30
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=np.zeros(4), ubu=np.full(4, 65.0)), max_batch=B)
    d = m.gen_inputs(B, seed=1004, ref='hover')
    m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
    torch.cuda.synchronize()
    t = (ctypes.c_int32 * (128 * 20))()
    assert m.lib.mpcb_debug_ref_trace(t) == 0
    a = np.frombuffer(t, dtype=np.uint32).reshape(128, 4, 5)
    for p in range(128):
        if not a[p].any():
            continue
        print(f'pass {p}: ' + ' | '.join(f'm{m_} lo {a[p, m_, 0]:08x} hi {a[p, m_, 1]:08x} rel {a[p, m_, 2]:08x} '
                                         f'+lo {a[p, m_, 3]:08x} +hi {a[p, m_, 4]:08x}' for m_ in range(4)))


if __name__ == '__main__':
    main()
