#!/usr/bin/env python3
"""B = 1 per-step latency of the c1 shape (12/4, N = 10, fp64, hover; BASELINE configs[0]) on each
solve path a handle can select (mpcb_capi.hip select_path): the default fused row kernel + the
16-lane forward pass, the two-launch form (MPCB_FUSE_P12=0), the small-chunk path with the
stage-parallel linearisation (MPCB_SMALL_MAX) and the single-kernel solver
(MPCB_SPLIT_MIN_BATCH).  Device-resident inputs, synchronised after every step, as
mpc_blaster_amd/latency.py measures c1_device_ms; u0 of every path against the default's.

    python tools/c1_paths.py [--n 400] [--N 10]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = [('default', {}), ('two launches', {'MPCB_FUSE_P12': '0'}),
            ('small-chunk', {'MPCB_SMALL_MAX': '64'}), ('single kernel', {'MPCB_SPLIT_MIN_BATCH': '2'})]
KEYS = ('MPCB_FUSE_P12', 'MPCB_SMALL_MAX', 'MPCB_SPLIT_MIN_BATCH')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=400)
    ap.add_argument('--N', type=int, default=10)
    args = ap.parse_args()
    import torch

    from mpc_blaster_amd.api import BatchedMPC
    from mpc_blaster_amd.config import MPCConfig
    from mpc_blaster_amd.latency import _timed
    x0 = np.array([[0.3, -0.2, 0.1, 0.05, -0.04, 0.1, 0.2, 0.1, -0.1, 0.02, -0.01, 0.03]])
    dev = lambda a: torch.as_tensor(a, dtype=torch.float64, device=0)  # noqa: E731
    dx0, dxr, dur = dev(x0), dev(np.zeros((1, args.N + 1, 12))), dev(np.full((1, args.N, 4), 22.0725))
    ref = None
    for name, env in VARIANTS:
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        m = BatchedMPC(MPCConfig(N=args.N, dtype='f64'), max_batch=1, device=0)
        med, p99 = _timed(lambda: m.solve(dx0, dxr, dur), args.n)
        u0 = m.get_control().cpu().numpy()
        ref = u0 if ref is None else ref
        print(f'{name:14s} {m.path:>6s}: c1 device {med * 1e3:7.1f} us (p99 {p99 * 1e3:7.1f}), '
              f'u0 vs default {np.abs(u0 - ref).max():.1e}, kernels {list(m.last_kernels().values())}',
              flush=True)
        m.close()
    for k in KEYS:
        os.environ.pop(k, None)
    # where the default path's time goes: the facade call, the bare C ABI call with its arguments
    # built once, and the C ABI call without a synchronisation after every step
    m = BatchedMPC(MPCConfig(N=args.N, dtype='f64'), max_batch=1, device=0)
    m.solve(dx0, dxr, dur)
    p = m._ptr
    cargs = (m._h, 1, p(dx0), 12, p(dxr), 0, p(dur), 0, p(None), 0, p(m._u0), p(m._X), p(m._U), p(m._status),
             m._stream())
    raw = lambda: m.lib.mpcb_solve(*cargs)  # noqa: E731
    med, p99 = _timed(raw, args.n)
    print(f'C ABI call alone (arguments built once): {med * 1e3:7.1f} us (p99 {p99 * 1e3:7.1f})', flush=True)
    reps = 20
    med, _ = _timed(lambda: [raw() for _ in range(reps)], max(args.n // reps, 5))
    print(f'C ABI calls back to back, one synchronisation per {reps}: {med * 1e3 / reps:7.1f} us per step', flush=True)
    med, _ = _timed(lambda: torch.cuda.synchronize(), args.n)
    print(f'synchronisation of an idle device alone: {med * 1e3:7.1f} us', flush=True)
    m.close()


if __name__ == '__main__':
    main()
