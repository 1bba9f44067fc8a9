#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of the three c2 kernels (variant built with -DMPCB_STAMPS).

    MPCB_LIB=mpc_blaster_amd/variants/lib_stamps.so python tools/wave_times.py

Each wave of P1 (row rollout), P2 (Riccati) and P3 (fwd_rm) records s_memrealtime (100 MHz) at
entry, loop start, loop end and exit (mpcb_common.h WT); printed in microseconds relative to the
kernel's first wave entry: the dispatch ramp (spread of entries), the prologue, loop and epilogue
medians, and the tail (spread of exits).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig, _lib  # noqa: E402

B, N = 4096, 20
m = BatchedMPC(MPCConfig(N=N, dtype='f64'), max_batch=B)
d = m.gen_inputs(B, seed=1002, ref='hover')
for _ in range(5):
    m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
torch.cuda.synchronize()
lib = _lib.load()
lib.mpcb_debug_wt_max.restype = ctypes.c_int
WMAX = lib.mpcb_debug_wt_max()   # table stride (mpcb_common.h MPCB_WT_MAX)
waves = B // 4
starts = {}
# (c2 runs P1 inside row_riccati_kernel: its table is p1f; MPCB_FUSE_P12=0 builds: p1)
for name in ('p1f' if os.environ.get('WT_P1', 'p1f') == 'p1f' else 'p1', 'p2', 'p3'):
    buf = (ctypes.c_ulonglong * (WMAX * 7))()
    f = getattr(lib, f'mpcb_debug_wt_{name}')
    name = name[:2]
    f.argtypes = [ctypes.c_void_p]
    assert f(buf) == 0
    raw = np.array(buf, dtype=np.uint64)
    hw = raw[WMAX * 4:WMAX * 4 + waves]
    t = raw[:WMAX * 4].astype(np.float64).reshape(WMAX, 4)[:waves] * 0.01   # us
    t0 = t[:, 0].min()
    starts[name] = (t0, t[:, 3].max())
    r = t - t0
    print(f'{name}: span {r[:, 3].max():6.2f} us | entries {np.percentile(r[:, 0], 50):5.2f} '
          f'(max {r[:, 0].max():5.2f}) | prologue {np.median(r[:, 1] - r[:, 0]):5.2f} | loop '
          f'{np.median(r[:, 2] - r[:, 1]):6.2f} (min {np.min(r[:, 2] - r[:, 1]):6.2f} max '
          f'{np.max(r[:, 2] - r[:, 1]):6.2f}) | epilogue {np.median(r[:, 3] - r[:, 2]):5.2f} | '
          f'exits p50 {np.percentile(r[:, 3], 50):6.2f} max {r[:, 3].max():6.2f}')
    if name == 'p2':
        lp = r[:, 2] - r[:, 1]
        hid = hw & 0xFFFFFFFF
        simd = (hid >> 4) & 3
        cu = (hid >> 8) & 15
        sh = (hid >> 12) & 1
        se = (hid >> 13) & 7
        xcc = (hw >> 32) & 15
        key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        share = cnt[inv]   # waves of this kernel on the same SIMD
        print('   p2 waves per SIMD: ', np.bincount(share).tolist(), '| loop median when alone',
              round(float(np.median(lp[share == 1])), 2), 'shared',
              round(float(np.median(lp[share > 1])), 2) if (share > 1).any() else None)
        xcd = np.arange(waves) % 8
        print('   p2 loop by blockIdx % 8:', ' '.join(f'{np.median(lp[xcd == x]):5.2f}' for x in range(8)),
              '| slowest 5% by XCD:', np.bincount(xcd[lp > np.percentile(lp, 95)], minlength=8).tolist())
        print('   p2 loop vs entry order: corr', round(float(np.corrcoef(lp, r[:, 0])[0, 1]), 3),
              '| vs P1 exit of the same quad: corr', round(float(np.corrcoef(lp, p1ex)[0, 1]), 3))
    if name == 'p1':
        p1ex = r[:, 3]
print(f'gaps: p1 end -> p2 first entry {starts["p2"][0] - starts["p1"][1]:5.2f} us, '
      f'p2 end -> p3 first entry {starts["p3"][0] - starts["p2"][1]:5.2f} us')
