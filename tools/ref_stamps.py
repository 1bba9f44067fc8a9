"""Diagnostic (GPU box): where the fp32 refinement kernel's time goes at c4.  Runs the c4 solve on
a MPCB_REF_STAMPS build (python tools/build_variant.py refst -DMPCB_REF_STAMPS=1; MPCB_LIB points
at it) and prints, per refinement call of workgroup 0, the s_memtime cycles of each sweep:
re-simulation, adjoint for the correction, correction backward, correction forward, deciding
adjoint.

    MPCB_LIB=$PWD/mpc_blaster_amd/variants/lib_refst.so python tools/ref_stamps.py [--solves 10]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--solves', type=int, default=10)
    a = ap.parse_args()
    import torch

    from mpc_blaster_amd import BatchedMPC, MPCConfig
    B, N = 65536, 30
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=np.zeros(4), ubu=np.full(4, 65.0)), max_batch=B)
    d = m.gen_inputs(B, seed=1004, ref='hover')
    m.solve(d['x0'], d['xref'], d['uref'])
    torch.cuda.synchronize()
    f = m.lib.mpcb_debug_ref_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = (ctypes.c_ulonglong * 8)()
    f(out, 1)
    for _ in range(a.solves):
        m.solve(d['x0'], d['xref'], d['uref'])
    torch.cuda.synchronize()
    f(out, 0)
    v = np.array(out[:8], dtype=np.float64)
    calls = max(v[5], 1)
    names = ['re-simulation', 'adjoint (correction)', 'correction backward', 'correction forward', 'adjoint (decide)']
    print(f'{int(v[5])} refinement calls in workgroup 0 over {a.solves} solves (N = {N})')
    for i, n in enumerate(names):
        print(f'  {n:22s} {v[i] / calls:10.0f} cycles per call, {v[i] / calls / N:7.0f} per stage')
    print(f'  total                  {v[:5].sum() / calls:10.0f} cycles per call')


if __name__ == '__main__':
    main()
