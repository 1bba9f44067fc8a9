#!/usr/bin/env python3
"""A/B of the c4 active-set kernel's work order (needs the MPCB_AS_ORDER_DBG variant:
tools/build_variant.py asord -DMPCB_AS_ORDER_DBG).  The work counter hands instances out in
index order; here the order comes from a previous solve's own pass counts (mpcb_qp_stats), most
passes first -- the longest-processing-time-first bound of any predictor -- against the index
order and a random one, with the outputs checked bit-identical across orders.

    MPCB_LIB=mpc_blaster_amd/variants/lib_asord.so python tools/ab_as_order.py [reps]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig, _lib  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, N = 65536, 30
m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=np.zeros(4), ubu=np.full(4, 65.0)), max_batch=B)
lib = _lib.load()
lib.mpcb_debug_set_as_order.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
d = m.gen_inputs(B, seed=1004, ref='hover', wind=False)
outs = {}


def run(name, order):
    lib.mpcb_debug_set_as_order(m._h, None if order is None else order.data_ptr())
    for _ in range(3):
        m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
    torch.cuda.synchronize()
    m.set_timing(True)
    ph = []
    for _ in range(REPS):
        m.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
        ph.append(m.last_timing())
    m.set_timing(False)
    torch.cuda.synchronize()
    fw = np.array([p['forward'] for p in ph])
    tot = np.array([sum(p.values()) for p in ph])
    outs[name] = [t.clone() for t in (m._u0, m._X, m._U, m._status)]
    print(f'{name:10s} active-set kernel {fw.mean():.4f} ms (min {fw.min():.4f}) | phases sum {tot.mean():.4f} ms',
          flush=True)
    return m.qp_stats(B)[:, 0].clone()


passes = run('index', None)
p = passes.cpu().numpy()
print(f'passes per instance: mean {p.mean():.2f} max {p.max()} (>8: {(p > 8).sum()})', flush=True)
lpt = torch.from_numpy(np.argsort(-p, kind='stable').astype(np.int32)).cuda()
rnd = torch.from_numpy(np.random.default_rng(0).permutation(B).astype(np.int32)).cuda()
rev = torch.flip(lpt, [0]).contiguous()
run('lpt', lpt)
run('random', rnd)
run('spt', rev)
# the hard instances first (longest first among them), the rest in index order (its locality)
hard = {}
for thr in (5, 6, 8):
    h = np.nonzero(p > thr)[0]
    h = h[np.argsort(-p[h], kind='stable')]
    rest = np.nonzero(p <= thr)[0]
    hard[thr] = torch.from_numpy(np.concatenate([h, rest]).astype(np.int32)).cuda()
    run(f'hard>{thr}', hard[thr])
# a predictor available before the active set: the unconstrained solution's box violation
# (the same P2 gains and forward pass as the active set's first pass), largest first for the
# top fraction, the rest in index order
mu = BatchedMPC(MPCConfig(N=N, dtype='f32'), max_batch=B)
mu.solve(d['x0'], d['xref'], d['uref'], want_traj=True)
Uu = mu._U.double()
mag = ((-Uu).clamp(min=0) + (Uu - 65.0).clamp(min=0)).sum(dim=(1, 2)).cpu().numpy()
nv = ((Uu < 0) | (Uu > 65.0)).sum(dim=(1, 2)).cpu().numpy()
mu.close()
for nm, key in (('mag', mag), ('nv', nv)):
    for frac in (0.03, 0.1):
        kth = np.sort(key)[::-1][int(frac * B)]
        h = np.nonzero(key > kth)[0]
        h = h[np.argsort(-key[h], kind='stable')]
        rest = np.nonzero(key <= kth)[0]
        o = torch.from_numpy(np.concatenate([h, rest]).astype(np.int32)).cuda()
        cap = (p[h] > 8).sum()
        print(f'{nm} top {frac:.0%}: {len(h)} first, {cap} of {(p > 8).sum()} hard (>8 passes) among them')
        run(f'{nm}{int(frac * 100)}', o)
run('index2', None)
run('lpt2', lpt)
for k in ('lpt', 'random', 'spt', 'hard>5', 'hard>6', 'hard>8', 'mag3', 'mag10', 'nv3', 'nv10', 'index2', 'lpt2'):
    same = all(torch.equal(a, b) for a, b in zip(outs['index'], outs[k]))
    print(f'{k}: outputs bit-identical to index order: {same}')
lib.mpcb_debug_set_as_order(m._h, None)
