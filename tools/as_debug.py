#!/usr/bin/env python3
"""Debug: the c4 active-set kernels (MPCB_AS=1 DPP / 0 LDS) on the same inputs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dt = sys.argv[2] if len(sys.argv) > 2 else 'f32'
N = 30
cfg = MPCConfig(N=N, dtype=dt, lbu=np.zeros(4), ubu=np.full(4, 65.0))
res = {}
for impl in ('1', '0'):
    os.environ['MPCB_AS'] = impl
    m = BatchedMPC(cfg, max_batch=B)
    d = m.gen_inputs(B, seed=1004, ref='hover')
    m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
    torch.cuda.synchronize()
    res[impl] = dict(U=m.get_input_trajectory().double().cpu().numpy(), st=m.get_status().cpu().numpy(),
                     qs=m.qp_stats(B).cpu().numpy(), x0=d['x0'].double().cpu().numpy())
a, b = res['1'], res['0']
oob = lambda U: ((U < -1e-4) | (U > 65 + 1e-3)).reshape(B, -1).any(1)
da = np.abs(a['U'] - b['U']).reshape(B, -1).max(1)
print('status!=0 new/old', (a['st'] != 0).sum(), (b['st'] != 0).sum())
print('out of bounds new/old', oob(a['U']).sum(), oob(b['U']).sum())
print('instances differing > 1e-4:', (da > 1e-4).sum(), 'max diff', da.max())
bad = np.nonzero(da > 1e-4)[0][:10]
print('first bad', bad, 'wave', bad // 4)
for i in bad[:5]:
    print(i, 'qstats new', a['qs'][i], 'old', b['qs'][i])
    print('   U new k:', np.nonzero(np.abs(a['U'][i] - b['U'][i]).max(1) > 1e-4)[0])
    print('   new', a['U'][i][:4], '\n   old', b['U'][i][:4])
ib = np.nonzero(oob(a['U']))[0]
if len(ib):
    from oracle.ocp import OcpSpec, mpc_solve
    for i in ib[:3]:
        Ui = a['U'][i]
        print('OOB instance', i, 'min', Ui.min(), 'max', Ui.max(), 'old min/max', b['U'][i].min(), b['U'][i].max())
        x0 = a['x0'][i:i + 1]
        o = mpc_solve(x0, np.tile(np.array([0, 0, 3.5] + [0] * 9, float) * 0, (1, N + 1, 1)) if False else None, None, None) if False else None
