#!/usr/bin/env python3
"""Diagnostic: per-region cycles of the Riccati stage loop (variant built with -DMPCB_STAMPS).

    MPCB_LIB=mpc_blaster_amd/variants/lib_stamps.so python tools/stamps.py [c2|c3]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig, _lib  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else 'c2'
B, dt, ref = {'c2': (4096, 'f64', 'hover'), 'c3': (65536, 'f32', 'sine'), 'c4': (65536, 'f32', 'hover')}[w]
N = 30 if w == 'c4' else 20
box = dict(lbu=np.zeros(4), ubu=np.full(4, 65.0)) if w == 'c4' else {}
m = BatchedMPC(MPCConfig(N=N, dtype=dt, **box), max_batch=B)
d = m.gen_inputs(B, seed=1004 if w == 'c4' else 1002, ref=ref)
for _ in range(3):
    m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
torch.cuda.synchronize()
lib = _lib.load()
out = (ctypes.c_ulonglong * 16)()
lib.mpcb_debug_stamps.argtypes = [ctypes.c_void_p]
assert lib.mpcb_debug_stamps(out) == 0
names = ['prefetch', 'tangent', 'export+Lv/X+sync', 'products', 'stagecost+Hu+syncs', 'chol+solves',
         'Pn', 'KR store+sync', 'publish+commit+sync', 'Pc select+LP']
v = np.array(out[:10], dtype=np.float64) / N
print(f'{w}: cycles per stage (s_memtime units, wave 0):')
for n, x in zip(names, v):
    print(f'   {n:24s} {x:9.0f}')
print(f'   {"total":24s} {v.sum():9.0f}')
v1 = np.array(out[13:16], dtype=np.float64) / N
print(f'{w}: P1 (nominal_quad) cycles per stage (wave 0):')
for n, x in zip(['u load + xu puts', 'rk4_nom (4 f + capture puts)', 'flush + syncs'], v1):
    print(f'   {n:32s} {x:9.0f}')
print(f'   {"total":32s} {v1.sum():9.0f}')

if hasattr(lib, 'mpcb_debug_stamps_as') and w == 'c4' and os.environ.get('MPCB_AS', '1') != '0':
    ob = (ctypes.c_ulonglong * 12)()
    lib.mpcb_debug_stamps_as.argtypes = [ctypes.c_void_p]
    assert lib.mpcb_debug_stamps_as(ob) == 0
    v = np.array(ob[:], dtype=np.float64)
    its, bst = v[8], v[9]
    nf = its * N
    print(f'c4 active-set kernel v2 (mpcb_as.hip), wave 0: {its:.0f} iterations, {bst:.0f} backward stages')
    print(f'   backward init per pass                 {v[0] / max(its - 1, 1):9.0f}')
    for n, x in zip(['bwd: loads, h, products, stage cost', 'bwd: input block, masking, Cholesky, P, stores',
                     'bwd: P transpose, snapshot'], v[1:4]):
        print(f'   {n:44s} {x / max(bst, 1):9.0f}   per backward stage')
    for n, x in zip(['fwd: prefetch issue', 'fwd: du, outputs', 'fwd: row dot, multiplier checks'], v[4:7]):
        print(f'   {n:44s} {x / nf:9.0f}   per forward stage')
    print(f'   {"fwd copy + tail + active-set updates":44s} {v[7] / its:9.0f}   per iteration')
    print(f'   total {v[:8].sum():.0f}')
elif hasattr(lib, 'mpcb_debug_stamps_box') and w == 'c4':
    ob = (ctypes.c_ulonglong * 12)()
    lib.mpcb_debug_stamps_box.argtypes = [ctypes.c_void_p]
    assert lib.mpcb_debug_stamps_box(ob) == 0
    v = np.array(ob[:], dtype=np.float64)
    its, bst = v[8], v[9]
    print(f'c4 active-set kernel, wave 0: {its:.0f} iterations, {bst:.0f} backward stages')
    print(f'   backward cycles per stage           {v[5] / max(bst, 1):9.0f}   (total {v[5]:.0f})')
    nf = its * N
    for n, x in zip(['fwd: regs (+prefetch wait)', 'fwd: fload issue', 'fwd: du dot', 'fwd: publish du, read z',
                     'fwd: outputs + dots + checks'], v[:5]):
        print(f'   {n:36s} {x / nf:9.0f}   per forward stage')
    print(f'   forward tail per pass               {v[6] / its:9.0f}')
    print(f'   active-set update per iteration     {v[7] / its:9.0f}')
    print(f'   total                               {v[:8].sum():9.0f}')
elif hasattr(lib, 'mpcb_debug_stamps_as') and w == 'c2':
    ob = (ctypes.c_ulonglong * 12)()
    lib.mpcb_debug_stamps_as.argtypes = [ctypes.c_void_p]
    assert lib.mpcb_debug_stamps_as(ob) == 0
    v = np.array(ob[:], dtype=np.float64) / N
    print(f'{w}: 16-lane DPP forward (fwd_rm_kernel) cycles per stage (wave 0):')
    for n, x in zip(['row assembly (+ slot wait)', 'du, outputs', 'row dot, refill issue'], v[4:7]):
        print(f'   {n:36s} {x:9.0f}')
    print(f'   {"total":36s} {v[4:7].sum():9.0f}')
elif hasattr(lib, 'mpcb_debug_stamps_box'):
    ob = (ctypes.c_ulonglong * 12)()
    lib.mpcb_debug_stamps_box.argtypes = [ctypes.c_void_p]
    if lib.mpcb_debug_stamps_box(ob) == 0:
        vb = np.array(ob[:5], dtype=np.float64) / N
        print(f'{w}: P3 (16-lane forward) cycles per stage (wave 0):')
        for n, x in zip(['stage start -> regs (+prefetch wait)', 'fload issue', 'du dot', 'publish du, read z', 'outputs + state dot'], vb):
            print(f'   {n:36s} {x:9.0f}')
        print(f'   {"total":36s} {vb.sum():9.0f}')
