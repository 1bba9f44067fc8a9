#!/usr/bin/env python3
"""12/4 input box: the active set with its interior-point fallback (default max_as_iter) against
the interior point from the start (max_as_iter = 1: every instance whose unconstrained solution
leaves the box goes straight to mpcb_asipm.h), on the c4 bench draws and on strongly constrained
iterate-mode draws (sine references, the iterate perturbed by 0.05 / 1 N; tests/test_gpu_fuzz.py
case 27's kind).  Device time per solve (HIP events) and the difference of the two solutions.

    python tools/box_ipm_direct.py [--B 65536]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import BatchedMPC, MPCConfig  # noqa: E402


def run(B, N, inp, iterate, cap, reps=10):
    m = BatchedMPC(MPCConfig(N=N, dtype='f32', lbu=np.zeros(4), ubu=np.full(4, 65.0), max_as_iter=cap), max_batch=B)
    args = [torch.as_tensor(inp[k], dtype=torch.float32, device='cuda') for k in ('x0', 'xref', 'uref')]
    it = [torch.as_tensor(inp[k], dtype=torch.float32, device='cuda') for k in ('xbar', 'ubar')] if iterate else None

    def solve():
        if iterate:
            m.solve_iterate(args[0], it[0], it[1], args[1], args[2])
        else:
            m.solve(args[0], args[1], args[2])
    for _ in range(2):
        solve()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        solve()
    e1.record()
    torch.cuda.synchronize()
    st = m.get_status().cpu().numpy()
    qs = m.qp_stats(B).cpu().numpy()
    return e0.elapsed_time(e1) / reps, m.get_input_trajectory().cpu().numpy().copy(), st, qs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=65536)
    B = ap.parse_args().B
    cases = {}
    gen = lambda N, seed, ref: {k: (None if v is None else v.double().cpu().numpy()) for k, v in
                                BatchedMPC(MPCConfig(N=N), max_batch=B).gen_inputs(B, seed=seed, ref=ref).items()}
    inp = gen(30, 1004, 'hover')
    cases['c4 bench draws (N = 30, rollout)'] = (30, inp, False)
    N = 11
    rng = np.random.default_rng(5)
    inp = gen(N, 1003, 'sine')
    inp['xbar'] = inp['xref'] + rng.normal(scale=0.05, size=(B, N + 1, 12))
    inp['ubar'] = inp['uref'] + rng.normal(scale=1.0, size=(B, N, 4))
    cases['strongly constrained (N = 11, iterate)'] = (N, inp, True)
    dump = {}
    for name, (N, inp, iterate) in cases.items():
        out = {}
        for cap in (200, 1):
            ms, U, st, qs = run(B, N, inp, iterate, cap)
            out[cap] = U
            print(f'{name}, max_as_iter {cap:3d}: {ms:7.3f} ms per solve, status {np.bincount(st, minlength=5).tolist()}, '
                  f'passes + interior-point iterations per instance: mean {qs[:, 0].mean():.1f} max {qs[:, 0].max()}',
                  flush=True)
        d = np.abs(out[200] - out[1]).max(axis=(1, 2)) / np.maximum(np.abs(out[1]).max(axis=(1, 2)), 1.0)
        print(f'  max normwise difference of U between the two: {d.max():.2e} (median {np.median(d):.1e})', flush=True)
        w = np.argsort(-d)[:8]   # the instances that differ most, for a CPU check against the oracle
        tag = 'c4' if N == 30 else 'sc'
        dump.update({f'{tag}_idx': w, f'{tag}_U_as': out[200][w], f'{tag}_U_ipm': out[1][w]})
        dump.update({f'{tag}_{k}': inp[k][w] for k in inp if inp[k] is not None and inp[k].shape[0] == B})
    os.makedirs('gpurun_out', exist_ok=True)
    np.savez('gpurun_out/box_ipm_direct_worst.npz', **dump)


if __name__ == '__main__':
    main()
