#!/usr/bin/env python3
"""Diagnostic: per-wave timeline of the fp32 Riccati kernel (riccati_kernel_f32, P2) at c3 / c5,
launch by launch, to find where its run-to-run spread comes from (round-4 verdict item 3).
Needs a variant built with -DMPCB_STAMPS (tools/build_variant.py stamps -DMPCB_STAMPS):

    MPCB_LIB=mpc_blaster_amd/variants/lib_stamps.so python tools/wave_times_p2.py [c3|c5] [launches]

Each P2 wave records s_memrealtime (100 MHz) at entry, loop start, loop end and exit plus its
HW_ID / XCC_ID (mpcb_common.h WT).  Per launch: the span, the waves each SIMD ran and the
spread of that count, the per-SIMD busy time (sum of its waves' entry->exit, overlaps merged),
the median and tail of the loop time, concurrency (waves resident per SIMD at mid-kernel), and
which XCD / SIMD finished last.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig, _lib  # noqa: E402

W = sys.argv[1] if len(sys.argv) > 1 else 'c3'
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B, N, ref, wind = {'c3': (65536, 20, 'sine', False), 'c5': (131072, 40, 'hover', True)}[W]
chunk = 65536   # one P2 launch per chunk (mpcb_create); the table holds the last launch
m = BatchedMPC(MPCConfig(N=N, dtype='f32'), max_batch=B)
d = m.gen_inputs(B, seed=1003 if W == 'c3' else 1005, ref=ref, wind=wind)
lib = _lib.load()
lib.mpcb_debug_wt_max.restype = ctypes.c_int
WMAX = lib.mpcb_debug_wt_max()
waves = min(B, chunk) // 4
assert waves <= WMAX
f = lib.mpcb_debug_wt_p2
f.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * (WMAX * 7))()
for _ in range(3):
    m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'], want_traj=W == 'c3')
torch.cuda.synchronize()
print(f'{W}: B={B} N={N}, P2 waves per launch {waves}')
for rep in range(REPS):
    m.set_timing(True)
    m.solve(d['x0'], d['xref'], d['uref'], wind=d['wind'], want_traj=W == 'c3')
    ph = m.last_timing()
    m.set_timing(False)
    torch.cuda.synchronize()
    assert f(buf) == 0
    raw = np.array(buf, dtype=np.uint64)
    hw = raw[WMAX * 4:WMAX * 4 + waves]
    t = raw[:WMAX * 4].astype(np.float64).reshape(WMAX, 4)[:waves] * 0.01   # us
    r = t - t[:, 0].min()
    hid = hw & 0xFFFFFFFF
    simd = (hid >> 4) & 3
    cu = (hid >> 8) & 15
    sh = (hid >> 12) & 1
    se = (hid >> 13) & 7
    xcc = (hw >> 32) & 15
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    ukey, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    loop = r[:, 2] - r[:, 1]
    cyc = (raw[WMAX * 6:WMAX * 6 + waves].astype(np.float64) - raw[WMAX * 5:WMAX * 5 + waves].astype(np.float64))
    mhz = cyc / np.maximum(loop, 1e-3)   # shader-clock cycles per microsecond of each wave's loop
    life = r[:, 3] - r[:, 0]
    span = r[:, 3].max()
    # per-SIMD: its last exit and the sum of its waves' lifetimes
    last = np.zeros(len(ukey))
    np.maximum.at(last, inv, r[:, 3])
    busy = np.zeros(len(ukey))
    np.add.at(busy, inv, life)
    mid = span / 2
    conc = np.zeros(len(ukey))
    np.add.at(conc, inv, ((r[:, 0] <= mid) & (r[:, 3] >= mid)).astype(float))
    ilast = int(np.argmax(r[:, 3]))
    kx = xcc.astype(int)
    xend = [float(r[kx == x, 3].max()) if (kx == x).any() else 0.0 for x in range(8)]
    print(f'launch {rep}: P2 {ph["riccati"] * 1e3 / max(1, -(-B // chunk)):7.1f} us/launch (events) | span {span:6.1f} us | '
          f'SIMDs {len(ukey)} waves/SIMD min {cnt.min()} med {int(np.median(cnt))} max {cnt.max()} | '
          f'loop med {np.median(loop):5.1f} p95 {np.percentile(loop, 95):5.1f} max {loop.max():5.1f} | '
          f'life med {np.median(life):5.1f} | SIMD last-exit p50 {np.median(last):6.1f} min {last.min():6.1f} | '
          f'resident at mid {np.bincount(conc.astype(int)).tolist()} | last wave: xcc {int(xcc[ilast])} '
          f'simd-waves {int(cnt[inv[ilast]])} entry {r[ilast, 0]:6.1f}')
    print(f'    clock (s_memtime / s_memrealtime over each loop) MHz: median {np.median(mhz):6.0f} '
          f'p5 {np.percentile(mhz, 5):6.0f} p95 {np.percentile(mhz, 95):6.0f} | loop cycles median {np.median(cyc):8.0f} '
          f'p95 {np.percentile(cyc, 95):8.0f} | by XCD MHz: ' + ' '.join(f'{np.median(mhz[kx == x]):5.0f}' for x in range(8)))
    print('    XCD last exit: ' + ' '.join(f'{v:6.1f}' for v in xend) +
          ' | entries p50 by XCD: ' + ' '.join(f'{np.median(r[kx == x, 0]):6.1f}' for x in range(8)))
